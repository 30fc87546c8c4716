"""ORACLE (test infrastructure only): the float64 restatement of oracle/nets_f64.py in torch
ops, so that a large-batch check (the CNN actor-critic at 4,096 samples per minibatch, 16
optimizer steps per train step, BASELINE configs[3]) runs on the test GPU in float64
instead of for minutes in numpy. Same layer semantics (xagents/utils/common.py:169-290):

* Dense: y = x @ W + b, W (in, out) (common.py:239-258);
* Conv1D (valid padding, common.py:231-237) on (B, H, W, C): along W with H folded into
  the batch, kernel (k, C_in, F), im2col column index t*C + c exactly as nets_f64;
* Flatten row-major over (H, W', F) (common.py:259-260);
* relu / tanh / linear (softmax outputs as logits).

The parameter gradient comes from torch autograd through these float64 ops (the ReLU
derivative at 0 is 0, as nets_f64's `y > 0`). tests/test_oracle.py pins this module
against nets_f64 on the CPU; only tests/ import it.
"""
import torch

from nets_f64 import param_slices


def _act(name, z):
    if name == 'relu':
        return torch.relu(z)
    if name == 'tanh':
        return torch.tanh(z)
    assert name in (None, 'linear', 'softmax'), name
    return z


def forward(layers, theta, x, input_shape, gates=None):
    """theta: flat float64 tensor (may require grad); x: uint8 or float tensor [B, ...].
    Returns (x as float64, [every layer's output]). gates {layer: bool tensor of the layer's
    output shape}: those ReLU layers take the given gate pattern instead of z > 0 (y = z
    where the gate is on, 0 elsewhere, and the same mask in the gradient) -- the f64 replay
    of a device run adopts the device's gates, which differ from the f64 forward's only at
    pre-activations within f32 rounding of zero (nets_f64.adopt_gates)."""
    gates = gates or {}

    def act(i, name, z):
        if i in gates:
            assert name == 'relu', name
            return z * gates[i].reshape(z.shape).to(z.dtype)
        return _act(name, z)

    if x.dtype == torch.uint8:
        x = (x.float() / 255.0).double()  # f32(u8) / 255 as the device loader, then f64
    else:
        x = x.double()
    B = x.shape[0]
    x = x.reshape(B, *input_shape)
    sls, _ = param_slices(layers)
    outs = []
    for i, l in enumerate(layers):
        src = x if l.input_index == -1 else outs[l.input_index]
        if l.kind == 'flatten':
            outs.append(src.reshape(B, -1))
            continue
        (o1, s1), (o2, s2) = sls[i]
        n1 = 1
        for d in s1:
            n1 *= d
        W = theta[o1:o1 + n1].reshape(s1)
        b = theta[o2:o2 + s2[0]]
        if l.kind == 'dense':
            outs.append(act(i, l.activation, src.reshape(B, -1) @ W + b))
        else:
            H, Win, C = src.shape[1:]
            k, s = l.size, l.stride
            P = (Win - k) // s + 1
            idx = (torch.arange(P, device=x.device)[:, None] * s
                   + torch.arange(k, device=x.device)[None, :])
            cols = src.reshape(B * H, Win, C)[:, idx, :].reshape(B * H, P, k * C)
            y = cols @ W.reshape(k * C, l.filters) + b
            outs.append(act(i, l.activation, y).reshape(B, H, P, l.filters))
    return x, outs


def gradient(layers, theta, x, input_shape, d_outputs):
    """Flat float64 parameter gradient for d(loss)/d(output) of the output layers
    ({layer index: tensor}), through a fresh forward at theta."""
    th = theta.detach().double().clone().requires_grad_(True)
    _, outs = forward(layers, th, x, input_shape)
    idx = sorted(d_outputs)
    g, = torch.autograd.grad([outs[i] for i in idx], [th],
                             grad_outputs=[d_outputs[i].reshape(outs[i].shape).double()
                                           for i in idx])
    return g
