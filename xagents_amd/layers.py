"""Device executor for .cfg-defined models (Conv1D / flatten / dense), the CNN and
wide-MLP path of the off-policy agents and the CNN actor-critic
(xagents/utils/common.py:169-290 builds the same graphs with Keras).

Every layer runs as one `xa_gemm` (gemm.hip) with grouped-affine operand addressing:
Conv1D on (B, H, W, C) input (conv along W, H folded into the batch)
is an implicit-im2col GEMM, its weight gradient the same GEMM with the im2col moved to
the reduction index, its input gradient one implicit transposed-conv GEMM
(`xa_conv1d_dgrad`; a dY W^T GEMM + fixed-order col2im gather, `xa_conv1d_input_grad`,
when the filter count is not a multiple of 4). Biases, ReLU / tanh and the ReLU gate of the backward
pass are GEMM epilogues. The NatureCNN stack (three Conv1D layers over 84 x 84 x 1 frames)
runs forward as one fused launch out of LDS (`xa_conv_stack_fwd`, conv_stack.hip). Image inputs stay uint8 in HBM and are scaled f32(x) / 255 in
the GEMM loader (xagents/base.py:505-506).

Buffers are allocated per batch size and reused; all launches go to torch's current
stream (graph-capturable).
"""
import functools
import os

import torch

from xagents_amd import _lib
from xagents_amd._lib import (XA_ACT_NONE, XA_ACT_RELU, XA_ACT_TANH, XaAdamApply,
                              XaConvStackArgs, XaConvStackBwdArgs, XaGemmArgs, call, stream)

_FORCE = int(os.environ.get('XA_GEMM_FORCE', '0'))
# algorithmic FLOPs per frame row of the NatureCNN conv stack (2 x MACs): forward conv1 +
# conv2 + conv3 = 2 (20 x 32 x 8 + 9 x 64 x 128 + 7 x 64 x 192); backward = every layer's
# weight gradient (= its forward) + the input gradients of conv2 and conv3
STACK_FWD_FLOPS = 2 * (20 * 32 * 8 + 9 * 64 * 128 + 7 * 64 * 192)
STACK_BWD_FLOPS = STACK_FWD_FLOPS + 2 * (9 * 64 * 128 + 7 * 64 * 192)
_ACTS = {None: XA_ACT_NONE, 'linear': XA_ACT_NONE, 'relu': XA_ACT_RELU, 'tanh': XA_ACT_TANH}


def act_code(name):
    if name not in _ACTS:
        raise NotImplementedError(f'activation {name!r} has no device epilogue')
    return _ACTS[name]


def _gemm_args(M, N, K, a, b, c, *, a_u8=False, a_m=(1, 0, 0), a_k=(1, 1, 0), b_ks, b_ns,
               ldc, bias=None, act=XA_ACT_NONE, gate=None, ld_gate=0, beta=False, workspace=None,
               splits=None, force_small=False, a_ones_row=False):
    lib = _lib.load()
    s = splits if splits is not None else lib.xa_gemm_splits(M, N, K)
    g = XaGemmArgs()
    g.M, g.N, g.K = int(M), int(N), int(K)
    ip = lambda v: None if v is None else int(v)  # noqa: E731  (numpy ints -> pointers)
    a, b, c, bias, gate = ip(a), ip(b), ip(c), ip(bias), ip(gate)
    g.a = a
    g.a_u8 = int(a_u8)
    g.a_pm, g.a_rm, g.a_sm = a_m
    g.a_pk, g.a_rk, g.a_sk = a_k
    g.b, g.b_ks, g.b_ns = b, b_ks, b_ns
    g.c, g.ldc = c, ldc
    g.splits = s
    if s > 1:
        need = s * M * N
        if workspace is None or workspace.numel() < need:
            raise _lib.HipLibraryError(f'xa_gemm: split workspace of {need} floats needed')
        g.partials = workspace.data_ptr()
    g.bias = bias
    g.act = act
    g.gate, g.ld_gate = gate, ld_gate
    g.beta = int(beta)
    # XA_GEMM_FORCE (diagnostic A/B): a force_small code for every call that passes none
    g.force_small = int(force_small) or _FORCE
    g.a_ones_row = int(a_ones_row)
    return g


def gemm(M, N, K, a, b, c, **kw):
    """C = [C +] act(A B + bias) * [gate > 0] with A(m, k) = a[f(m) + g(k)],
    f / g given as (group, row stride, in-group stride) triples (gemm.hip)."""
    call('xa_gemm', ctypes_ref(_gemm_args(M, N, K, a, b, c, **kw)), stream())


def gemm_adam(M, N, K, a, b, c, adam, **kw):
    """A weight-gradient GEMM with Keras Adam in its epilogue (xa_gemm_adam): `adam` an
    XaAdamApply over the parameters C is the gradient of; c = None writes no gradient."""
    call('xa_gemm_adam', ctypes_ref(_gemm_args(M, N, K, a, b, c, splits=1, **kw)),
         ctypes_ref(adam), stream())


def adam_apply(theta, m, v, step, opt, offset, grad_scale=1.0):
    """XaAdamApply of the parameters theta[offset:] (Keras Adam state m, v, iterations step
    of optimizer `opt`)."""
    from xagents_amd.kernels import _f32
    ad = XaAdamApply()
    offset = int(offset)
    ad.theta, ad.m, ad.v = theta.data_ptr() + 4 * offset, m.data_ptr() + 4 * offset, \
        v.data_ptr() + 4 * offset
    ad.step = step.data_ptr()
    ad.lr, ad.beta1, ad.beta2 = _f32(opt.learning_rate), _f32(opt.beta_1), _f32(opt.beta_2)
    ad.eps, ad.grad_scale = _f32(opt.epsilon), _f32(grad_scale)
    return ad


@functools.lru_cache(maxsize=None)
def fold_bias_ok(M, N, K):
    """A weight gradient [M, N] (K reduction rows) and its bias gradient can run as ONE GEMM
    with a constant-one row appended to A (a_ones_row: the 64 x 64 kernel the dispatcher
    picks for the few-row reductions of small batches); else two launches."""
    lib = _lib.load()
    return lib.xa_gemm_shape(M + 1, N, K, lib.xa_gemm_splits(M + 1, N, K)) == 0


def ctypes_ref(x):
    import ctypes
    return ctypes.byref(x)


class LayerExecutor:
    """Forward / backward of a DeviceModel's layer list at a fixed batch size."""

    def __init__(self, model, batch):
        self.model = model
        self.B = batch
        self.dev = model.theta.device
        self.layers = model.layers
        self.in_shape = tuple(model.input_shape)
        self.offsets = []
        off = 0
        for l in self.layers:
            if l.kind in ('dense', 'convolutional'):
                wn = (l.in_features * l.units if l.kind == 'dense'
                      else l.size * l.in_features * l.filters)
                bn = l.units if l.kind == 'dense' else l.filters
                self.offsets.append((off, off + wn))
                off += wn + bn
            else:
                self.offsets.append(None)
        assert off == model.n_params
        f32 = dict(dtype=torch.float32, device=self.dev)
        self.outs = [None if l.kind == 'flatten' else
                     torch.empty(batch, *l.out_shape, **f32) for l in self.layers]
        for i, l in enumerate(self.layers):
            if l.kind == 'flatten':
                self.outs[i] = self._src(i).reshape(batch, -1) if l.input_index != -1 else None
        self.douts = [None if l.kind == 'flatten' else torch.empty_like(self.outs[i])
                      for i, l in enumerate(self.layers)]
        ws = 0
        dcol = 0
        lib = _lib.load()
        for i, l in enumerate(self.layers):
            for (M, N, K) in self._gemm_shapes(i):
                s = lib.xa_gemm_splits(M, N, K)
                ws = max(ws, s * M * N if s > 1 else 0)
            if l.kind == 'convolutional' and l.input_index != -1 and not self._dgrad_ok(i):
                rows, P, kC = self._conv_dims(i)[0], self._conv_dims(i)[2], l.size * l.in_features
                dcol = max(dcol, rows * P * kC)
        self.workspace = torch.empty(max(ws, 1), **f32)
        self.dcol = torch.empty(max(dcol, 1), **f32)
        # narrow convs (k C <= 8): weight + bias gradient in one pass (xa_conv1d_wgrad)
        self.wg_floats = [int(lib.xa_conv1d_wgrad_workspace_floats(l.size, l.in_features, l.filters))
                          if l.kind == 'convolutional' else 0 for l in self.layers]
        self.wg_ws = torch.empty(max(self.wg_floats + [1]), **f32)
        self.stack = self._conv_stack()
        # the fused stack backward's per-workgroup partials (allocated on first use; executors
        # that run one at a time may share one, as they share `workspace`)
        self.stack_ws = None

    # the forward writes the conv stack's h1 / h2 (the backward's gates and weight-gradient
    # operands); forward-only executors (acting, target networks) may turn this off
    keep_hidden = True

    def _conv_stack(self):
        """True when layers 0-2 are the NatureCNN Conv1D stack over (84, 84, 1) frames
        (32 x 8 / 4, 64 x 4 / 2, 64 x 3 / 1, ReLU): the forward then runs them as one
        xa_conv_stack_fwd launch (XA_CONV_STACK=0: per-layer GEMMs)."""
        import os
        if os.environ.get('XA_CONV_STACK', '1') == '0' or len(self.layers) < 3:
            return False
        want = ((-1, 8, 4, 32, 1), (0, 4, 2, 64, 32), (1, 3, 1, 64, 64))
        for i, (src, k, st, f, c) in enumerate(want):
            l = self.layers[i]
            if (l.kind != 'convolutional' or l.input_index != src or l.size != k or
                    l.stride != st or l.filters != f or l.in_features != c or
                    self._act(i) != XA_ACT_RELU):
                return False
        return (tuple(self.in_shape[-3:]) == (84, 84, 1) and
                tuple(self.layers[2].out_shape[-2:]) == (7, 64) and
                all(self.offsets[i][0] % 4 == 0 for i in range(3)))

    def _conv_stack_fwd(self, x, tp):
        a = XaConvStackArgs()
        a.x, a.x_u8 = x.data_ptr(), int(x.dtype == torch.uint8)
        a.rows = self.B * self.in_shape[-3]
        (w1, b1), (w2, b2), (w3, b3) = ((int(u), int(v)) for u, v in self.offsets[:3])
        a.w1, a.b1, a.w2, a.b2 = tp + 4 * w1, tp + 4 * b1, tp + 4 * w2, tp + 4 * b2
        a.w3, a.b3 = tp + 4 * w3, tp + 4 * b3
        if self.keep_hidden:
            a.h1, a.h2 = self.outs[0].data_ptr(), self.outs[1].data_ptr()
        a.h3 = self.outs[2].data_ptr()
        ev = self._timing_start()
        call('xa_conv_stack_fwd', ctypes_ref(a), stream())
        self._timing_end(ev, f'conv stack fwd {a.rows} rows', float(STACK_FWD_FLOPS) * a.rows)

    def _conv_stack_bwd(self, Bb, gp, accumulate, adam=None):
        """Layers 2..0's parameter gradient in one fused launch + reduce (xa_conv_stack_bwd)
        from douts[2] (conv3's gated output gradient) and the forward's h1 / h2. adam
        (XaAdamApply of the stack's first parameter, keep_grad, rest): Keras Adam on the
        stack's parameters inside the reduce (the raw gradient to grad only when keep_grad),
        and rest = (XaAdamApply, gradient pointer, count) of one more range whose gradient
        is final by now, or None."""
        rows = Bb * self.in_shape[-3]
        lib = _lib.load()
        need = int(lib.xa_conv_stack_bwd_workspace_floats(int(self.B * self.in_shape[-3])))
        if self.stack_ws is None or self.stack_ws.numel() < need:
            self.stack_ws = torch.empty(need, dtype=torch.float32, device=self.dev)
        tp = self.model.theta.data_ptr()
        (w1, _), (w2, _), (w3, _) = ((int(u), int(v)) for u, v in self.offsets[:3])
        a = XaConvStackBwdArgs()
        a.x, a.x_u8, a.rows = self.x.data_ptr(), int(self.x.dtype == torch.uint8), int(rows)
        a.w2, a.w3 = tp + 4 * w2, tp + 4 * w3
        a.h1, a.h2, a.dz3 = (self.outs[0].data_ptr(), self.outs[1].data_ptr(),
                             self.douts[2].data_ptr())
        a.ws, a.ws_floats = self.stack_ws.data_ptr(), self.stack_ws.numel()
        a.grad, a.accumulate = (gp + 4 * w1 if gp is not None else None), int(accumulate)
        if adam is not None:
            ad, keep, rest = adam
            a.adam_on, a.write_grad, a.adam = 1, int(bool(keep)), ad
            if rest is not None:
                a.rest, a.rest_grad, a.n_rest = rest[0], int(rest[1]), int(rest[2])
        ev = self._timing_start()
        call('xa_conv_stack_bwd', ctypes_ref(a), stream())
        self._timing_end(ev, f'conv stack bwd {rows} rows (+ reduce)',
                         float(STACK_BWD_FLOPS) * rows)

    def _stack_bwd_ok(self):
        """The fused backward covers layers 0-2 when they are the stack, contiguous in theta
        ([w1 b1 w2 b2 w3 b3]), and the forward kept h1 / h2 (XA_CONV_STACK_BWD=0: per
        layer)."""
        if not self.stack or not self.keep_hidden or \
                os.environ.get('XA_CONV_STACK_BWD', '1') == '0':
            return False
        end = None
        for i in range(3):
            w0, b0 = self.offsets[i]
            l = self.layers[i]
            if end is not None and w0 != end:
                return False
            if b0 != w0 + l.size * l.in_features * l.filters:
                return False
            end = b0 + l.filters
        return True

    def _act(self, i):
        """Epilogue of layer i. A softmax output layer (the ACER actor,
        xagents/acer/models/cnn-actor-critic.cfg) yields its pre-softmax logits: the loss
        head applies the softmax and returns the gradient w.r.t. the logits."""
        name = self.layers[i].activation
        if name == 'softmax' and i in self.model.outputs:
            return XA_ACT_NONE
        return act_code(name)

    def adam_fusable(self, i, batch=None):
        """Dense layer i's [W; b] weight gradient can carry its Adam step (xa_gemm_adam: the
        64 x 64 kernel with the bias as a constant-one row, one K split, f32 input, 16-B
        aligned rows)."""
        l = self.layers[i]
        if l.kind != 'dense' or self._src_layer(i) == -1:
            return False
        Bb = batch or self.B
        w0, b0 = self.offsets[i]
        lib = _lib.load()
        n_in, n_out = l.in_features, l.units
        return (b0 == w0 + n_in * n_out and w0 % 4 == 0 and n_out % 4 == 0 and
                lib.xa_gemm_splits(n_in + 1, n_out, Bb) == 1 and
                lib.xa_gemm_shape(n_in + 1, n_out, Bb, 1) == 0)

    def _dgrad_ok(self, i):
        """xa_conv1d_dgrad needs F % 4 == 0 and a 16-byte aligned kernel slice."""
        return self.layers[i].filters % 4 == 0 and self.offsets[i][0] % 4 == 0

    # ---- optional per-launch timing (bench): HIP events on the launch stream ----
    timing = None  # a list to collect (name, start event, end event, flops) into

    def _timing_start(self):
        if self.timing is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _timing_end(self, e0, name, flops, nbytes=None):
        """(name, start, end, algorithmic FLOPs, algorithmic HBM bytes or None when the
        launch is MFMA-bound) -- bench.py's dominant-kernel roofline."""
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.timing.append((name, e0, e1, flops, nbytes))

    # ---- shapes --------------------------------------------------------------
    def _src_shape(self, i):
        l = self.layers[i]
        return self.in_shape if l.input_index == -1 else self.layers[l.input_index].out_shape

    def _src(self, i):
        j = self.layers[i].input_index
        while j != -1 and self.layers[j].kind == 'flatten':
            j = self.layers[j].input_index
        return None if j == -1 else self.outs[j]

    def _src_layer(self, i):
        """Index of the layer whose buffer feeds layer i (flatten resolved), or -1."""
        j = self.layers[i].input_index
        while j != -1 and self.layers[j].kind == 'flatten':
            j = self.layers[j].input_index
        return j

    def _conv_dims(self, i, batch=None):
        l = self.layers[i]
        H, Win, C = self._src_shape(i)[-3:]
        P = l.out_shape[-2]
        return (batch or self.B) * H, Win, P, C

    def _gemm_shapes(self, i):
        l = self.layers[i]
        B = self.B
        if l.kind == 'dense':
            return [(B, l.units, l.in_features), (l.in_features, l.units, B), (1, l.units, B),
                    (B, l.in_features, l.units), (l.in_features + 1, l.units, B)]
        if l.kind == 'convolutional':
            rows, Win, P, C = self._conv_dims(i)
            kC = l.size * C
            return [(rows * P, l.filters, kC), (kC, l.filters, rows * P),
                    (1, l.filters, rows * P), (rows * P, kC, l.filters),
                    (kC + 1, l.filters, rows * P)]
        return []

    # ---- forward ---------------------------------------------------------------
    def forward(self, x, head=None):
        """x: [B, *input_shape] uint8 (images) or f32. Returns the output layers' tensors.
        `head` (an XaDqnHeadArgs): the last layer, a row-dot-shaped Q head, runs as
        xa_dqn_head with DQN's per-row step (argmax or TD target + gradient) in its launch."""
        assert x.shape[0] == self.B and x.is_contiguous()
        theta = self.model.theta
        tp = theta.data_ptr()
        u8 = x.dtype == torch.uint8
        self.x = x
        if self.stack:
            self._conv_stack_fwd(x, tp)
        fused_head = self._fused_head_layer()
        for i, l in enumerate(self.layers):
            if l.kind == 'flatten' or (self.stack and i < 3) or i == fused_head:
                continue
            j = self._src_layer(i)
            src = x if j == -1 else self.outs[j]
            src_u8 = u8 and j == -1
            w0, b0 = self.offsets[i]
            if l.kind == 'dense':
                ev = self._timing_start()
                kw = dict(a_u8=src_u8, a_m=(1, l.in_features, 0), b_ks=l.units, b_ns=1,
                          ldc=l.units, bias=tp + 4 * b0, act=self._act(i),
                          workspace=self.workspace)
                if fused_head is not None and i == fused_head - 1:
                    # this layer's split reduce, the head and (head given) DQN's row step in
                    # one launch after the split partials (xa_gemm_head)
                    lh = self.layers[fused_head]
                    wh, bh = self.offsets[fused_head]
                    gd = _gemm_args(self.B, l.units, l.in_features, src.data_ptr(), tp + 4 * w0,
                                    self.outs[i].data_ptr(), **kw)
                    gh = _gemm_args(self.B, lh.units, lh.in_features, self.outs[i].data_ptr(),
                                    tp + 4 * wh, self.outs[fused_head].data_ptr(),
                                    a_m=(1, lh.in_features, 0), b_ks=lh.units, b_ns=1,
                                    ldc=lh.units, bias=tp + 4 * bh, act=self._act(fused_head),
                                    workspace=self.workspace)
                    call('xa_gemm_head', ctypes_ref(gd), ctypes_ref(gh),
                         None if head is None else ctypes_ref(head), stream())
                    self._timing_end(ev, f'dense fwd {self.B}x{l.units}x{l.in_features} + head',
                                     2.0 * self.B * (l.units * l.in_features +
                                                     lh.units * lh.in_features))
                    continue
                if head is not None and i == len(self.layers) - 1:
                    g = _gemm_args(self.B, l.units, l.in_features, src.data_ptr(), tp + 4 * w0,
                                   self.outs[i].data_ptr(), **kw)
                    call('xa_dqn_head', ctypes_ref(g), ctypes_ref(head), stream())
                else:
                    gemm(self.B, l.units, l.in_features, src.data_ptr(), tp + 4 * w0,
                         self.outs[i].data_ptr(), **kw)
                self._timing_end(ev, f'dense fwd {self.B}x{l.units}x{l.in_features}',
                                 2.0 * self.B * l.units * l.in_features)
            else:
                rows, Win, P, C = self._conv_dims(i)
                gemm(rows * P, l.filters, l.size * C, src.data_ptr(), tp + 4 * w0,
                     self.outs[i].data_ptr(), a_u8=src_u8, a_m=(P, Win * C, l.stride * C),
                     b_ks=l.filters, b_ns=1, ldc=l.filters, bias=tp + 4 * b0,
                     act=self._act(i), workspace=self.workspace)
        return [self.outs[i] for i in self.model.outputs]

    def _head_bwd_on(self):
        """xa_head_bwd for row-dot heads (XA_HEAD_BWD=0: the dW GEMM + few-k dX launches)."""
        if '_hb' not in self.__dict__:
            self._hb = os.environ.get('XA_HEAD_BWD', '1') != '0'
        return self._hb

    def _fused_head_layer(self):
        """The index of the model's single output layer when it is a row-dot head on the
        dense layer right before it and that pair takes xa_gemm_head (one launch for the
        dense layer's split reduce and the head); None otherwise (XA_GEMM_HEAD=0: never)."""
        if '_fh' not in self.__dict__:
            fh = None
            h = len(self.layers) - 1
            if os.environ.get('XA_GEMM_HEAD', '1') != '0' and h >= 1 and \
                    list(self.model.outputs) == [h] and self.layers[h].kind == 'dense' and \
                    self.layers[h - 1].kind == 'dense' and self._src_layer(h) == h - 1 and \
                    self._src_layer(h - 1) != -1:
                l, lh = self.layers[h - 1], self.layers[h]
                tp = self.model.theta.data_ptr()
                (w0, b0), (wh, bh) = self.offsets[h - 1], self.offsets[h]
                src = self.outs[self._src_layer(h - 1)]
                try:
                    gd = _gemm_args(self.B, l.units, l.in_features, src.data_ptr(), tp + 4 * w0,
                                    self.outs[h - 1].data_ptr(), a_m=(1, l.in_features, 0),
                                    b_ks=l.units, b_ns=1, ldc=l.units, bias=tp + 4 * b0,
                                    act=self._act(h - 1), workspace=self.workspace)
                    gh = _gemm_args(self.B, lh.units, lh.in_features, self.outs[h - 1].data_ptr(),
                                    tp + 4 * wh, self.outs[h].data_ptr(),
                                    a_m=(1, lh.in_features, 0), b_ks=lh.units, b_ns=1,
                                    ldc=lh.units, bias=tp + 4 * bh, act=self._act(h),
                                    workspace=self.workspace)
                    if _lib.load().xa_gemm_head_ok(ctypes_ref(gd), ctypes_ref(gh)) == 1:
                        fh = h
                except _lib.HipLibraryError:
                    fh = None
            self._fh = fh
        return self._fh

    # ---- forward-mode derivative ------------------------------------------------
    def jvp(self, v):
        """Tangents of the output layers along the flat parameter direction `v` (Keras
        variable order) at the last forward's input: per layer dz = x dW + dx W + db,
        dy = act'(y) dz, i.e. J v for TRPO's Fisher-vector product (the R-operator of the
        double tape in xagents/trpo/agent.py:121-148). Returns [B, n] tensors."""
        if getattr(self, 'touts', None) is None:
            self.touts = [None if l.kind == 'flatten' else torch.empty_like(self.outs[i])
                          for i, l in enumerate(self.layers)]
            for i, l in enumerate(self.layers):
                if l.kind == 'flatten':
                    j = self._src_layer(i)
                    self.touts[i] = None if j == -1 else self.touts[j].reshape(self.B, -1)
        tp, vp = self.model.theta.data_ptr(), v.data_ptr()
        u8 = self.x.dtype == torch.uint8
        for i, l in enumerate(self.layers):
            if l.kind == 'flatten':
                continue
            j = self._src_layer(i)
            src = self.x if j == -1 else self.outs[j]
            tsrc = None if j == -1 else self.touts[j]
            src_u8 = u8 and j == -1
            w0, b0 = self.offsets[i]
            out = self.touts[i]
            if l.kind == 'dense':
                geo = dict(a_m=(1, l.in_features, 0), b_ks=l.units, b_ns=1, ldc=l.units)
                M, N, K = self.B, l.units, l.in_features
            else:
                rows, Win, P, C = self._conv_dims(i)
                geo = dict(a_m=(P, Win * C, l.stride * C), b_ks=l.filters, b_ns=1,
                           ldc=l.filters)
                M, N, K = rows * P, l.filters, l.size * C
            # x dW + db, then + dx W (the input tangent, absent for the model input)
            gemm(M, N, K, src.data_ptr(), vp + 4 * w0, out.data_ptr(), a_u8=src_u8,
                 bias=vp + 4 * b0, workspace=self.workspace, **geo)
            if tsrc is not None:
                gemm(M, N, K, tsrc.data_ptr(), tp + 4 * w0, out.data_ptr(), beta=True,
                     workspace=self.workspace, **geo)
            a = self._act(i)
            if a != XA_ACT_NONE:
                call('xa_activation_grad', self.outs[i].data_ptr(), out.data_ptr(), out.numel(),
                     a, out.data_ptr(), stream())
        return [self.touts[i] for i in self.model.outputs]

    # ---- backward ----------------------------------------------------------------
    def backward(self, d_outputs, grad, batch=None, dinput=None, accumulate=False,
                 on_grad=None, adam=None):
        """d_outputs: gradients w.r.t. the output layers (model.outputs order, [b, n]).
        Writes the flat parameter gradient into `grad` (Keras variable order; None skips
        the parameter gradients) and, if given, d(loss)/d(input) into `dinput` [b, in]
        (dense input layers). `batch` (<= B) back-propagates only the first rows of the
        last forward (samples are independent rows, so a prefix of every buffer is a
        smaller batch). `accumulate` adds the parameter gradient to `grad` (chunked
        minibatches). `on_grad(w0)` is called once the launches writing a layer's weight
        and bias gradient (flat offsets w0 ..) are queued, before its input gradient's:
        layers finish in reverse order, so grad[w0:] is then final (the hook of the
        data-parallel path's bucketed all-reduce). `adam` {layer index: (XaAdamApply,
        keep_grad)}: those dense layers (adam_fusable) take their Keras Adam step inside the
        weight-gradient GEMM (xa_gemm_adam) after their input gradient has read W; `grad`
        then receives their raw gradient only when keep_grad. adam['stack'] (see
        _conv_stack_bwd): the fused conv stack's Adam (+ one more final range) inside its
        reduce launch."""
        Bb = batch or self.B
        assert adam is None or not accumulate
        assert Bb <= self.B
        # a forward-only executor's fused conv-stack forward never wrote h1 / h2, which the
        # backward reads as gates and weight-gradient operands
        if not (self.keep_hidden or not self.stack):
            raise RuntimeError('LayerExecutor.backward: this executor runs the fused conv '
                               'stack forward-only (keep_hidden=False); its hidden '
                               'activations are not materialised')
        tp = self.model.theta.data_ptr()
        gp = grad.data_ptr() if grad is not None else None
        written = [False] * len(self.layers)
        dz = {}
        for i, d in zip(self.model.outputs, d_outputs):
            l = self.layers[i]
            a = self._act(i)
            if a == XA_ACT_NONE:
                dz[i] = d.contiguous()
            else:
                out = self.douts[i]
                call('xa_activation_grad', self.outs[i].data_ptr(), d.contiguous().data_ptr(),
                     d.numel(), a, out.data_ptr(), stream())
                dz[i] = out
        u8 = self.x.dtype == torch.uint8
        for i in range(len(self.layers) - 1, -1, -1):
            l = self.layers[i]
            if l.kind == 'flatten':
                continue
            if i not in dz:
                if not written[i]:
                    continue
                # hidden layer: its ReLU gate was applied by the consumers (gate=out);
                # a tanh hidden layer takes the derivative here
                if self._act(i) == XA_ACT_TANH:
                    call('xa_activation_grad', self.outs[i].data_ptr(),
                         self.douts[i].data_ptr(), self.douts[i][:Bb].numel(), XA_ACT_TANH,
                         self.douts[i].data_ptr(), stream())
                dz[i] = self.douts[i]
            d = dz[i]
            if i == 2 and gp is not None and self._stack_bwd_ok():
                # the whole conv stack at once; layers finish in reverse order as below
                self._conv_stack_bwd(Bb, gp, accumulate,
                                     adam.get('stack') if adam is not None else None)
                if on_grad is not None:
                    for k in (2, 1, 0):
                        on_grad(self.offsets[k][0])
                break
            j = self._src_layer(i)
            src = self.x if j == -1 else self.outs[j]
            src_u8 = u8 and j == -1
            w0, b0 = self.offsets[i]
            gate_j = None
            if j != -1 and self._act(j) == XA_ACT_RELU:
                gate_j = self.outs[j].data_ptr()
            if l.kind == 'dense':
                n_in, n_out = l.in_features, l.units
                fused = adam is not None and i in adam

                def wgrad():
                    ev = self._timing_start()
                    if fused:
                        # [W; b] gradient + the layer's Adam step in one launch; reads W's
                        # old value nowhere (the input gradient below ran first)
                        ad, keep = adam[i]
                        gemm_adam(n_in + 1, n_out, Bb, src.data_ptr(), d.data_ptr(),
                                  gp + 4 * w0 if keep else None, ad, a_m=(1, 1, 0),
                                  a_k=(1, n_in, 0), b_ks=n_out, b_ns=1, ldc=n_out,
                                  a_ones_row=True)
                    elif gp is not None:
                        # dW = X^T dZ ; db = 1^T dZ -- one GEMM into the contiguous [W; b]
                        # block (b0 = w0 + n_in n_out) when the 64 x 64 kernel takes it
                        fold = fold_bias_ok(n_in, n_out, Bb) and b0 == w0 + n_in * n_out
                        gemm(n_in + fold, n_out, Bb, src.data_ptr(), d.data_ptr(), gp + 4 * w0,
                             a_u8=src_u8, a_m=(1, 1, 0), a_k=(1, n_in, 0), b_ks=n_out, b_ns=1,
                             ldc=n_out, beta=accumulate, workspace=self.workspace,
                             a_ones_row=fold)
                        if not fold:
                            gemm(1, n_out, Bb, None, d.data_ptr(), gp + 4 * b0, a_m=(1, 0, 0),
                                 a_k=(1, 0, 0), b_ks=n_out, b_ns=1, ldc=n_out, beta=accumulate,
                                 workspace=self.workspace)
                    if fused:
                        # HBM-bound: theta, m, v read + written (24 B per parameter), X, dZ
                        self._timing_end(ev, f'dense dW+Adam {n_in}x{n_out}x{Bb}',
                                         2.0 * (n_in + 1) * n_out * Bb,
                                         24.0 * (n_in + 1) * n_out + 4.0 * Bb * (n_in + n_out))
                    elif gp is not None:
                        self._timing_end(ev, f'dense dW {n_in}x{n_out}x{Bb}',
                                         2.0 * (n_in + 1) * n_out * Bb)
                    if gp is not None and on_grad is not None:
                        on_grad(w0)

                if not fused and gp is not None and j != -1 and n_out <= 8 and Bb <= 256 and \
                        n_in <= 4096 and not src_u8 and self._head_bwd_on():
                    # a row-dot head: its input gradient and [W; b] gradient in one launch
                    ev = self._timing_start()
                    call('xa_head_bwd', src.data_ptr(), d.data_ptr(), int(tp + 4 * w0),
                         None if gate_j is None else int(gate_j), int(Bb), int(n_in), int(n_out),
                         self.douts[j].data_ptr(), int(written[j]), int(gp + 4 * w0),
                         int(gp + 4 * b0), int(accumulate), stream())
                    self._timing_end(ev, f'head bwd {Bb}x{n_in}x{n_out}',
                                     4.0 * Bb * n_in * n_out)
                    written[j] = True
                    if on_grad is not None:
                        on_grad(w0)
                    continue
                if not fused:
                    wgrad()
                if j == -1 and dinput is not None:
                    gemm(Bb, n_in, n_out, d.data_ptr(), tp + 4 * w0, dinput.data_ptr(),
                         a_m=(1, n_out, 0), b_ks=1, b_ns=n_out, ldc=n_in,
                         workspace=self.workspace)
                if j != -1:
                    # dX = dZ W^T (gated by the source layer's ReLU), accumulated over heads
                    ev = self._timing_start()
                    gemm(Bb, n_in, n_out, d.data_ptr(), tp + 4 * w0,
                         self.douts[j].data_ptr(), a_m=(1, n_out, 0), b_ks=1, b_ns=n_out,
                         ldc=n_in, gate=gate_j, ld_gate=n_in if gate_j else 0,
                         beta=written[j], workspace=self.workspace)
                    self._timing_end(ev, f'dense dX {Bb}x{n_in}x{n_out}', 2.0 * Bb * n_in * n_out)
                    written[j] = True
                if fused:
                    wgrad()
            else:
                rows, Win, P, C = self._conv_dims(i, Bb)
                k, s, F = l.size, l.stride, l.filters
                if gp is not None and self.wg_floats[i]:
                    call('xa_conv1d_wgrad', src.data_ptr(), int(src_u8), d.data_ptr(),
                         int(rows), int(Win), int(C), int(P), int(k), int(s), int(F),
                         int(gp + 4 * w0), int(gp + 4 * b0), int(accumulate),
                         self.wg_ws.data_ptr(), self.wg_floats[i], stream())
                elif gp is not None:
                    fold = fold_bias_ok(k * C, F, rows * P) and b0 == w0 + k * C * F
                    gemm(k * C + fold, F, rows * P, src.data_ptr(), d.data_ptr(), gp + 4 * w0,
                         a_u8=src_u8, a_m=(1, 1, 0), a_k=(P, Win * C, s * C), b_ks=F, b_ns=1,
                         ldc=F, beta=accumulate, workspace=self.workspace, a_ones_row=fold)
                    if not fold:
                        gemm(1, F, rows * P, None, d.data_ptr(), gp + 4 * b0, a_m=(1, 0, 0),
                             a_k=(1, 0, 0), b_ks=F, b_ns=1, ldc=F, beta=accumulate,
                             workspace=self.workspace)
                if gp is not None and on_grad is not None:
                    on_grad(w0)
                if j != -1:
                    assert not written[j], 'a conv input with two consumers is not supported'
                    if self._dgrad_ok(i):
                        # implicit transposed-conv GEMM straight into dX (no im2col buffer)
                        call('xa_conv1d_dgrad', d.data_ptr(), int(tp + 4 * w0), int(rows),
                             int(P), int(k), int(s), int(C), int(F), int(Win), gate_j,
                             self.douts[j].data_ptr(), stream())
                    else:
                        gemm(rows * P, k * C, F, d.data_ptr(), tp + 4 * w0,
                             self.dcol.data_ptr(), a_m=(1, F, 0), b_ks=1, b_ns=F, ldc=k * C,
                             workspace=self.workspace)
                        call('xa_conv1d_input_grad', self.dcol.data_ptr(), rows, P, k, s, C,
                             Win, gate_j, self.douts[j].data_ptr(), stream())
                    written[j] = True
        return grad
