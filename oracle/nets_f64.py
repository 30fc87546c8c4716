"""ORACLE (test infrastructure only): float64 numpy restatement of the Keras layers the
reference's .cfg models are built from (xagents/utils/common.py:169-290):

* Dense: y = x @ W + b, W shape (in, out) (common.py:239-258);
* Conv1D (valid padding, common.py:231-237) applied to rank-4 (B, H, W, C) input: the
  convolution runs along W with H folded into the batch; kernel (k, C_in, F);
* Flatten: row-major over (H, W', F) (common.py:259-260);
* activations relu / tanh / linear (softmax outputs as logits).

`forward` returns every layer output; `backward` takes d(loss)/d(output) for each
output layer and returns the flat parameter gradient in Keras trainable_variables
order (kernel, bias per layer). Image inputs are scaled f32(u8) / 255 first
(xagents/base.py:505-506). Only tests/ import this module.
"""
import numpy as np


def _act(name, z):
    if name == 'relu':
        return np.maximum(z, 0.0)
    if name == 'tanh':
        return np.tanh(z)
    # a softmax output layer yields its pre-softmax logits (the ACER actor): the loss
    # restatement applies the softmax, as the device executor does
    assert name in (None, 'linear', 'softmax'), name
    return z


def _act_grad(name, y, dy):
    if name == 'relu':
        return dy * (y > 0)
    if name == 'tanh':
        return dy * (1.0 - y * y)
    return dy


def param_slices(layers):
    out, off = [], 0
    for l in layers:
        if l.kind == 'dense':
            shapes = [(l.in_features, l.units), (l.units,)]
        elif l.kind == 'convolutional':
            shapes = [(l.size, l.in_features, l.filters), (l.filters,)]
        else:
            out.append(None)
            continue
        sl = []
        for s in shapes:
            n = int(np.prod(s))
            sl.append((off, s))
            off += n
        out.append(sl)
    return out, off


def _weights(theta, sl):
    (o1, s1), (o2, s2) = sl
    return (theta[o1:o1 + int(np.prod(s1))].reshape(s1).astype(np.float64),
            theta[o2:o2 + int(np.prod(s2))].reshape(s2).astype(np.float64))


def _im2col(x, k, s):
    """x (R, W, C) -> (R, P, k*C) with column index t*C + c."""
    R, W, C = x.shape
    P = (W - k) // s + 1
    idx = np.arange(P)[:, None] * s + np.arange(k)[None, :]
    return x[:, idx, :].reshape(R, P, k * C)


def forward(layers, theta, x, input_shape):
    """Layer outputs (list, one per layer, batch-first)."""
    x = np.asarray(x)
    if x.dtype == np.uint8:
        x = (x.astype(np.float32) / np.float32(255.0)).astype(np.float64)
    else:
        x = x.astype(np.float64)
    B = x.shape[0]
    x = x.reshape(B, *input_shape)
    sls, _ = param_slices(layers)
    outs = []
    for i, l in enumerate(layers):
        src = x if l.input_index == -1 else outs[l.input_index]
        if l.kind == 'flatten':
            outs.append(src.reshape(B, -1))
        elif l.kind == 'dense':
            W, b = _weights(theta, sls[i])
            outs.append(_act(l.activation, src.reshape(B, -1) @ W + b))
        else:
            W, b = _weights(theta, sls[i])
            H, Win, C = src.shape[1:]
            cols = _im2col(src.reshape(B * H, Win, C), l.size, l.stride)
            y = cols @ W.reshape(l.size * C, l.filters) + b
            outs.append(_act(l.activation, y).reshape(B, H, cols.shape[1], l.filters))
    return x, outs


def backward(layers, theta, x_in, outs, d_outputs, want_input_grad=False, abs_terms=None,
             d_layers=None):
    """d_outputs: {layer index: d(loss)/d(layer output)} for the output layers.
    Returns the flat gradient, and d(loss)/d(input) too when want_input_grad.
    abs_terms: an optional [P] array that receives, per parameter, the sum of the absolute
    values of the terms its gradient sums (|x|^T |dz|, sum |dz|) -- the scale of the
    rounding error an f32 reduction of those terms can carry when they cancel."""
    sls, P = param_slices(layers)
    grad = np.zeros(P)
    B = x_in.shape[0]
    dys = {i: np.asarray(d, np.float64).reshape(outs[i].shape) for i, d in d_outputs.items()}
    dx = None
    for i in range(len(layers) - 1, -1, -1):
        if i not in dys:
            continue
        l = layers[i]
        if d_layers is not None:  # d(loss)/d(output) of every layer, for diagnostics
            d_layers[i] = dys[i]
        src = x_in if l.input_index == -1 else outs[l.input_index]
        if l.kind == 'flatten':
            dsrc = dys[i].reshape(src.shape)
        elif l.kind == 'dense':
            W, _ = _weights(theta, sls[i])
            dz = _act_grad(l.activation, outs[i], dys[i])
            xs = src.reshape(B, -1)
            (o1, s1), (o2, s2) = sls[i]
            grad[o1:o1 + W.size] += (xs.T @ dz).ravel()
            grad[o2:o2 + s2[0]] += dz.sum(0)
            if abs_terms is not None:
                abs_terms[o1:o1 + W.size] += (np.abs(xs).T @ np.abs(dz)).ravel()
                abs_terms[o2:o2 + s2[0]] += np.abs(dz).sum(0)
            dsrc = (dz @ W.T).reshape(src.shape)
        else:
            W, _ = _weights(theta, sls[i])
            H, Win, C = src.shape[1:]
            k, s = l.size, l.stride
            dz = _act_grad(l.activation, outs[i], dys[i])
            R = B * H
            Pn = dz.shape[2]
            dz2 = dz.reshape(R * Pn, l.filters)
            cols = _im2col(src.reshape(R, Win, C), k, s).reshape(R * Pn, k * C)
            (o1, s1), (o2, s2) = sls[i]
            grad[o1:o1 + W.size] += (cols.T @ dz2).ravel()
            grad[o2:o2 + s2[0]] += dz2.sum(0)
            if abs_terms is not None:
                abs_terms[o1:o1 + W.size] += (np.abs(cols).T @ np.abs(dz2)).ravel()
                abs_terms[o2:o2 + s2[0]] += np.abs(dz2).sum(0)
            dcol = (dz2 @ W.reshape(k * C, l.filters).T).reshape(R, Pn, k, C)
            dsrc = np.zeros((R, Win, C))
            for p in range(Pn):
                dsrc[:, p * s:p * s + k, :] += dcol[:, p]
            dsrc = dsrc.reshape(src.shape)
        if l.input_index != -1:
            j = l.input_index
            dys[j] = dys[j] + dsrc if j in dys else dsrc
        else:
            dx = dsrc if dx is None else dx + dsrc
    return (grad, dx) if want_input_grad else grad


def adopt_gates(layers, outs, device_outs, tol=1e-5):
    """Return a copy of the f64 layer outputs whose ReLU gates follow the device's f32
    forward (device_outs: {layer: array}), and the number of gates that differed. An
    f32 and an f64 forward disagree on a gate only where the pre-activation is ~0; each
    such flip moves one gradient element by its full value, so backward parity is checked
    with the device's own gates. Asserts that every flip sits within tol x the layer's
    largest output of zero."""
    outs = list(outs)
    flips = 0
    for i, l in enumerate(layers):
        if getattr(l, 'activation', None) != 'relu' or i not in device_outs:
            continue
        dev = np.asarray(device_outs[i]).reshape(outs[i].shape) > 0
        ref = outs[i] > 0
        bad = dev != ref
        if bad.any():
            scale = np.abs(outs[i]).max()
            assert (np.abs(np.asarray(device_outs[i], np.float64).reshape(outs[i].shape))[bad]
                    <= tol * scale).all(), f'layer {i}: a gate differs away from zero'
            flips += int(bad.sum())
            o = outs[i].copy()
            o[bad & dev] = np.finfo(np.float64).tiny
            o[bad & ~dev] = 0.0
            outs[i] = o
    return outs, flips

