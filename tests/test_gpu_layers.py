"""GPU parity of the GEMM building block and of .cfg models run by the layer executor
(xagents_amd/layers.py) against the float64 restatement (oracle/nets_f64.py).
Float tolerance: f32 accumulation vs f64, rtol 1e-4 relative to the output scale."""
import ctypes
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _close(got, ref, rtol=1e-4):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-12)
    err = np.abs(got - ref).max() / scale
    assert err < rtol, f'max error {err:.3g} (relative to max |ref| = {scale:.3g})'


# shapes reaching each kernel: small 64x64, square 128x128, tall 256x64, wide 64x256, and
# few-row many-split shapes (the batch-16/32/64 dense forward -- the split-K forward kernel
# for M <= 64, N % 64 == 0, K >= 8192; ragged M / N / K splits)
_SHAPES = [(37, 50, 29, 1), (64, 512, 3000, 8), (130, 70, 1000, 4), (300, 257, 400, 1),
           (1000, 40, 333, 2), (50, 700, 290, 3), (40, 50, 20000, 16), (200, 64, 17001, 1),
           (16, 512, 37632, 256), (5, 1000, 3001, 16), (32, 36, 8000, 64), (1, 512, 9000, 64),
           (17, 260, 5000, 32), (64, 512, 37632, 256), (32, 512, 37632, 256),
           (33, 448, 12345, 100),
           # few-column heads (row-dot path: N <= 8, K <= 4096)
           (64, 6, 512, 2), (128, 1, 512, 1), (3, 8, 4096, 4), (1000, 5, 77, 1),
           # few-k (elementwise path: K <= 8)
           (64, 512, 6, 1), (300, 64, 4, 1), (7, 9, 1, 1)]


@pytest.mark.parametrize('small', [False, True])
@pytest.mark.parametrize('M,N,K,splits', _SHAPES + [
    # few rows over a huge K (the NatureCNN dense forward at the acting batch)
    (32, 512, 37632, 256), (17, 448, 12345, 100),
    # the streaming path: two 512-column blocks, a 2-row-block M, a ragged K split
    (48, 1024, 20000, 128), (7, 512, 37632, 300)])
def test_gemm_plain_bias_relu_split(device, M, N, K, splits, small):
    from xagents_amd.layers import gemm
    from xagents_amd._lib import XA_ACT_RELU
    rng = np.random.default_rng(M + N + K)
    A = rng.normal(size=(M, K)).astype(np.float32)
    B = rng.normal(size=(K, N)).astype(np.float32)
    b = rng.normal(size=N).astype(np.float32)
    ta, tb, tbias = (torch.from_numpy(x).to(device) for x in (A, B, b))
    C = torch.empty(M, N, device=device)
    ws = torch.empty(splits * M * N + 1, device=device)
    gemm(M, N, K, ta.data_ptr(), tb.data_ptr(), C.data_ptr(), a_m=(1, K, 0), b_ks=N, b_ns=1,
         ldc=N, bias=tbias.data_ptr(), act=XA_ACT_RELU, workspace=ws, splits=splits,
         force_small=small)
    ref = np.maximum(A.astype(np.float64) @ B + b, 0)
    _close(C.cpu().numpy(), ref)


@pytest.mark.parametrize('M,N,K', [(64, 512, 6), (128, 37632, 4), (5, 3, 1)])
def test_gemm_head_input_gradient_few_k(device, M, N, K):
    """The heads' input gradient dX = dZ W^T with K = the head width (<= 8: the few-k path),
    the source layer's ReLU gate and beta accumulation (two heads into one dX), vs f64."""
    from xagents_amd.layers import gemm
    rng = np.random.default_rng(M + N + K)
    dZ = rng.normal(size=(M, K)).astype(np.float32)
    W = rng.normal(size=(N, K)).astype(np.float32)           # the head's [n_in, n_out] block^T
    gate = rng.normal(size=(M, N)).astype(np.float32)
    C0 = rng.normal(size=(M, N)).astype(np.float32)
    tdz, tw, tg = (torch.from_numpy(x).to(device) for x in (dZ, W, gate))
    C = torch.from_numpy(C0).to(device)
    gemm(M, N, K, tdz.data_ptr(), tw.data_ptr(), C.data_ptr(), a_m=(1, K, 0), b_ks=1, b_ns=K,
         ldc=N, gate=tg.data_ptr(), ld_gate=N, beta=True, workspace=torch.empty(1, device=device))
    ref = C0 + np.where(gate > 0, dZ.astype(np.float64) @ W.T, 0.0)
    _close(C.cpu().numpy(), ref)


@pytest.mark.parametrize('M,N,K,beta', [(512, 6, 64, False), (37632, 512, 64, False),
                                         (192, 64, 37632, True), (129, 70, 3001, False),
                                         (5, 7, 9, True)])
def test_gemm_ones_row_weight_and_bias_gradient(device, M, N, K, beta):
    """a_ones_row: the weight gradient X^T dZ [M, N] and the bias gradient 1^T dZ [N] of a
    layer as one GEMM into the contiguous [W; b] block (A = X^T read m-major with row M the
    constant 1), against float64; beta accumulates into both (chunked minibatches)."""
    from xagents_amd.layers import fold_bias_ok, gemm
    from xagents_amd import _lib
    assert fold_bias_ok(M, N, K)
    rng = np.random.default_rng(M + N + K)
    X = rng.normal(size=(K, M)).astype(np.float32)           # K rows of the layer input
    dZ = rng.normal(size=(K, N)).astype(np.float32)
    C0 = rng.normal(size=(M + 1, N)).astype(np.float32)
    tx, tdz = torch.from_numpy(X).to(device), torch.from_numpy(dZ).to(device)
    C = torch.from_numpy(C0).to(device)
    s = _lib.load().xa_gemm_splits(M + 1, N, K)
    ws = torch.empty(max(s, 1) * (M + 1) * N + 1, device=device)
    gemm(M + 1, N, K, tx.data_ptr(), tdz.data_ptr(), C.data_ptr(), a_m=(1, 1, 0),
         a_k=(1, M, 0), b_ks=N, b_ns=1, ldc=N, beta=beta, workspace=ws, a_ones_row=True)
    ref = np.concatenate([X.astype(np.float64).T @ dZ, dZ.astype(np.float64).sum(0)[None]])
    if beta:
        ref = ref + C0
    _close(C.cpu().numpy(), ref)


@pytest.mark.parametrize('M,N,K', [(37632, 512, 64), (128, 68, 33), (129, 68, 33),
                                   (3000, 512, 40), (64, 8, 100)])
def test_gemm_adam_is_gemm_then_adam_bit_for_bit(device, M, N, K):
    """xa_gemm_adam (the [W; b] weight gradient with Keras Adam in its epilogue, XCD-ordered
    1-D tile grid) against the gradient GEMM (same 64 x 64 kernel, one split) followed by
    xa_clip_adam with no clip: parameters, moments and the written raw gradient
    bit-identical; 2 chained steps so the second reads moments the first wrote. Covers the
    C3 shape (37632 x 512: 4712 tiles), ragged M / K, the scalar A loader (M + 1 = 130) and
    grids padded past the last row tile."""
    from xagents_amd import _lib, kernels
    from xagents_amd.layers import adam_apply, fold_bias_ok, gemm, gemm_adam
    if not fold_bias_ok(M, N, K):
        pytest.skip('shape not on the 64 x 64 kernel')
    rng = np.random.default_rng(M + N + K)
    X = torch.from_numpy(rng.normal(size=(K, M)).astype(np.float32)).to(device)
    dZ = torch.from_numpy(rng.normal(size=(K, N)).astype(np.float32)).to(device)
    th0 = rng.normal(size=(M + 1) * N).astype(np.float32)

    class Opt:
        learning_rate, beta_1, beta_2, epsilon = 1e-3, 0.9, 0.999, 1e-7

    kw = dict(a_m=(1, 1, 0), a_k=(1, M, 0), b_ks=N, b_ns=1, ldc=N, a_ones_row=True)
    res = []
    for fused in (False, True):
        th = torch.from_numpy(th0.copy()).to(device)
        m = torch.zeros_like(th)
        v = torch.zeros_like(th)
        step = torch.zeros(1, dtype=torch.int32, device=device)
        g = torch.empty_like(th)
        for _ in range(2):
            _lib.call('xa_adam_step_bump', step.data_ptr(), _lib.stream())
            if fused:
                gemm_adam(M + 1, N, K, X.data_ptr(), dZ.data_ptr(), g.data_ptr(),
                          adam_apply(th, m, v, step, Opt, 0), **kw)
            else:
                gemm(M + 1, N, K, X.data_ptr(), dZ.data_ptr(), g.data_ptr(), splits=1,
                     workspace=torch.empty(1, device=device), **kw)
                kernels.clip_adam(th, m, v, g, step, Opt.learning_rate, Opt.beta_1,
                                  Opt.beta_2, Opt.epsilon, clip_norm=0.0)
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in (th, m, v, g)])
    for a, b in zip(*res):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize('M,N,K', [(70, 45, 33), (260, 300, 77), (700, 60, 45), (60, 400, 50)])
def test_gemm_transposes_gate_beta_u8(device, M, N, K):
    from xagents_amd.layers import gemm
    rng = np.random.default_rng(3)
    At = rng.normal(size=(K, M)).astype(np.float32)      # A = At^T  (m-major loader)
    Bt = rng.normal(size=(N, K)).astype(np.float32)      # B = Bt^T  (k-major loader)
    gate = rng.normal(size=(M, N)).astype(np.float32)
    C0 = rng.normal(size=(M, N)).astype(np.float32)
    ta, tb, tg = (torch.from_numpy(x).to(device) for x in (At, Bt, gate))
    C = torch.from_numpy(C0.copy()).to(device)
    gemm(M, N, K, ta.data_ptr(), tb.data_ptr(), C.data_ptr(), a_m=(1, 1, 0), a_k=(1, M, 0),
         b_ks=1, b_ns=K, ldc=N, gate=tg.data_ptr(), ld_gate=N, beta=True, splits=1)
    ref = C0 + (At.T.astype(np.float64) @ Bt.T) * (gate > 0)
    _close(C.cpu().numpy(), ref)
    # uint8 A scaled by 1/255 (base.py:505-506), implicit Conv1D im2col: rows of W=20,
    # C=3 channels, kernel 4, stride 2 -> P = 9 positions
    rows, W, Cc, k, s = 11 + M // 10, 20, 3, 4, 2
    P = (W - k) // s + 1
    x = rng.integers(0, 256, size=(rows, W, Cc), dtype=np.uint8)
    Wt = rng.normal(size=(k * Cc, 8)).astype(np.float32)
    tx = torch.from_numpy(x).to(device)
    tw = torch.from_numpy(Wt).to(device)
    out = torch.empty(rows * P, 8, device=device)
    gemm(rows * P, 8, k * Cc, tx.data_ptr(), tw.data_ptr(), out.data_ptr(), a_u8=True,
         a_m=(P, W * Cc, s * Cc), b_ks=8, b_ns=1, ldc=8, splits=1)
    xf = (x.astype(np.float32) / np.float32(255.0)).astype(np.float64)
    idx = np.arange(P)[:, None] * s + np.arange(k)[None, :]
    cols = xf[:, idx, :].reshape(rows * P, k * Cc)
    _close(out.cpu().numpy(), cols @ Wt)


@pytest.mark.parametrize('M', [4, 64, 336])
def test_gemm_dense_input_gradient_shape(device, M):
    """dX = dZ W^T of the 37632 x 512 dense layer (B read k-major), split as the executor
    splits it, gated; relative to each row's scale."""
    from xagents_amd.layers import gemm
    from xagents_amd._lib import load
    N, K = 37632, 512
    rng = np.random.default_rng(M)
    dz = rng.normal(size=(M, K)).astype(np.float32)
    W = (rng.normal(size=(N, K)) * 0.01).astype(np.float32)   # (in, out) = Keras layout
    gate = rng.normal(size=(M, N)).astype(np.float32)
    s = load().xa_gemm_splits(M, N, K)
    tdz, tw, tg = (torch.from_numpy(x).to(device) for x in (dz, W, gate))
    C = torch.empty(M, N, device=device)
    ws = torch.empty(max(s, 1) * M * N + 1, device=device)
    gemm(M, N, K, tdz.data_ptr(), tw.data_ptr(), C.data_ptr(), a_m=(1, K, 0), b_ks=1,
         b_ns=K, ldc=N, gate=tg.data_ptr(), ld_gate=N, workspace=ws)
    ref = (dz.astype(np.float64) @ W.T.astype(np.float64)) * (gate > 0)
    got = C.cpu().numpy().astype(np.float64)
    err = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert err < 1e-6, f'splits {s}: relative error {err:.3g}'


@pytest.mark.parametrize('M,N,K', [(1, 2048, 256), (17, 2050, 768), (64, 4100, 512),
                                   (100, 2048, 256), (128, 3000, 1024), (200, 2064, 256),
                                   (384, 2048, 512), (336, 2100, 512), (33, 2048, 128),
                                   (64, 2064, 256)])
def test_gemm_small_m_kmajor(device, M, N, K):
    """The small-M kernel (both operands k-major, dX = dY W^T shapes): ragged M / N, K with
    and without the 2-wave K split, bias + ReLU, gate and beta accumulation vs float64."""
    from xagents_amd.layers import gemm
    from xagents_amd._lib import XA_ACT_RELU
    rng = np.random.default_rng(M * 7 + K)
    A = rng.normal(size=(M, K)).astype(np.float32)
    W = rng.normal(size=(N, K)).astype(np.float32)      # B(k, n) = W[n][k]
    bias = rng.normal(size=N).astype(np.float32)
    gate = rng.normal(size=(M, N)).astype(np.float32)
    C0 = rng.normal(size=(M, N)).astype(np.float32)
    ta, tw, tb, tg = (torch.from_numpy(x).to(device) for x in (A, W, bias, gate))
    C = torch.from_numpy(C0.copy()).to(device)
    gemm(M, N, K, ta.data_ptr(), tw.data_ptr(), C.data_ptr(), a_m=(1, K, 0), b_ks=1, b_ns=K,
         ldc=N, bias=tb.data_ptr(), act=XA_ACT_RELU, gate=tg.data_ptr(), ld_gate=N, beta=True,
         splits=1)
    z = np.maximum(A.astype(np.float64) @ W.T.astype(np.float64) + bias, 0)
    _close(C.cpu().numpy(), C0 + z * (gate > 0))


def _model(cfg, units, input_shape, device, seed=5):
    from xagents_amd.nets import Adam, ModelReader
    return ModelReader(str(cfg), units, input_shape, Adam(), seed=seed,
                       device=device).build_model()


@pytest.mark.parametrize('cfg,units,shape,B', [
    ('dqn/models/cnn.cfg', [6], (84, 84, 1), 2),
    ('dqn/models/cnn.cfg', [6], (84, 84, 1), 64),   # C3's batch: dense dX at M = 64
    ('ppo/models/cnn-actor-critic.cfg', [4, 1], (84, 84, 1), 3),
    ('td3/models/ann-actor.cfg', [4], (24,), 9),
    ('td3/models/ann-critic.cfg', [1], (28,), 9),
])
def test_layer_executor_forward_backward_vs_f64(device, cfg, units, shape, B):
    import sys
    sys.path.insert(0, str(ROOT / 'oracle'))
    import nets_f64 as O
    from xagents_amd.layers import LayerExecutor
    model = _model(ROOT / 'xagents_amd' / cfg, units, shape, device)
    rng = np.random.default_rng(11)
    if len(shape) == 3:
        x = rng.integers(0, 256, size=(B, *shape), dtype=np.uint8)
    else:
        x = rng.normal(size=(B, *shape)).astype(np.float32)
    ex = LayerExecutor(model, B)
    outs = ex.forward(torch.from_numpy(x).to(device))
    theta = model.theta.cpu().numpy()
    x64, ref_outs = O.forward(model.layers, theta, x, shape)
    for o, i in zip(outs, model.outputs):
        _close(o.cpu().numpy(), ref_outs[i])
    douts = [rng.normal(size=o.shape).astype(np.float32) for o in outs]
    grad = torch.zeros(model.n_params, device=device)
    ex.backward([torch.from_numpy(d).to(device) for d in douts], grad)
    # backward parity with the device's ReLU gates: an f32 / f64 disagreement on a gate
    # (pre-activation within 1e-5 of 0, asserted) moves one gradient element by its full
    # value, which is not an arithmetic error of the backward
    dev = {i: ex.outs[i].cpu().numpy() for i, l in enumerate(model.layers) if l.kind != 'flatten'}
    gated, flips = O.adopt_gates(model.layers, ref_outs, dev)
    print(f'{flips} gate flips')
    ref_g = O.backward(model.layers, theta, x64, gated,
                       {i: d for i, d in zip(model.outputs, douts)})
    # per parameter tensor, relative to that tensor's scale
    sls, _ = O.param_slices(model.layers)
    g = grad.cpu().numpy()
    for sl in sls:
        if sl is None:
            continue
        for off, s in sl:
            n = int(np.prod(s))
            _close(g[off:off + n], ref_g[off:off + n], rtol=2e-4)


@pytest.mark.parametrize('K,splits', [(100, 1), (50000, 64), (200000, 1024)])
def test_gemm_column_sums(device, K, splits):
    """A = NULL (ones) with M = 1: bias gradients (column sums of B)."""
    from xagents_amd.layers import gemm
    rng = np.random.default_rng(K)
    N = 70
    B = rng.normal(size=(K, N)).astype(np.float32)
    tb = torch.from_numpy(B).to(device)
    C = torch.zeros(1, N, device=device)
    ws = torch.empty(splits * N + 1, device=device)
    gemm(1, N, K, None, tb.data_ptr(), C.data_ptr(), b_ks=N, b_ns=1, ldc=N, workspace=ws,
         splits=splits)
    _close(C.cpu().numpy()[0], B.astype(np.float64).sum(0))


@pytest.mark.parametrize('rows,W,C,F,k,s', [
    (7, 20, 32, 64, 4, 2),    # NatureCNN conv2 input (BNT = 32 tiles, two phases)
    (5, 9, 64, 64, 3, 1),     # NatureCNN conv3 input (BNT = 64 tiles)
    (3, 24, 96, 8, 5, 2),     # k not a multiple of s, W_in past the last window, 2 channel tiles
    (4, 11, 17, 12, 2, 3),    # stride > kernel: phase 2 has no taps (all-zero rows)
    (130, 84, 32, 64, 8, 4),  # many rows, stride 4
])
def test_conv1d_dgrad_vs_f64_and_col2im(device, rows, W, C, F, k, s):
    """xa_conv1d_dgrad (implicit transposed-conv GEMM) against the f64 Conv1D input
    gradient and the two-launch path it replaces (dY W^T GEMM + xa_conv1d_input_grad)."""
    from xagents_amd._lib import call, stream
    from xagents_amd.layers import gemm
    rng = np.random.default_rng(rows * W + C)
    P = (W - k) // s + 1
    dy = rng.normal(size=(rows, P, F)).astype(np.float32)
    wk = rng.normal(size=(k, C, F)).astype(np.float32)
    gate = rng.normal(size=(rows, W, C)).astype(np.float32)
    ref = np.zeros((rows, W, C))
    for p in range(P):
        for t in range(k):
            ref[:, p * s + t, :] += dy[:, p, :].astype(np.float64) @ wk[t].T.astype(np.float64)
    ref_g = ref * (gate > 0)
    tdy, tw, tg = (torch.from_numpy(x).to(device) for x in (dy, wk, gate))
    for g_ptr, want in ((None, ref), (tg.data_ptr(), ref_g)):
        out = torch.full((rows, W, C), float('nan'), device=device)
        call('xa_conv1d_dgrad', tdy.data_ptr(), tw.data_ptr(), rows, P, k, s, C, F, W, g_ptr,
             out.data_ptr(), stream())
        torch.cuda.synchronize()
        _close(out.cpu().numpy(), want)
        # the im2col + col2im path (same math, different summation order)
        dcol = torch.empty(rows * P, k * C, device=device)
        gemm(rows * P, k * C, F, tdy.data_ptr(), tw.data_ptr(), dcol.data_ptr(),
             a_m=(1, F, 0), b_ks=1, b_ns=F, ldc=k * C, splits=1)
        out2 = torch.empty_like(out)
        call('xa_conv1d_input_grad', dcol.data_ptr(), rows, P, k, s, C, W, g_ptr,
             out2.data_ptr(), stream())
        torch.cuda.synchronize()
        _close(out.cpu().numpy(), out2.cpu().numpy().astype(np.float64))


@pytest.mark.parametrize('u8', [False, True])
@pytest.mark.parametrize('rows,W,C,k,s,F', [(50, 84, 1, 8, 4, 32), (7, 30, 2, 3, 2, 64),
                                             (3, 9, 1, 1, 1, 4)])
def test_conv1d_wgrad_small_vs_f64(device, rows, W, C, k, s, F, u8):
    """xa_conv1d_wgrad: one-pass dW + db of a narrow Conv1D vs float64, plain and
    accumulating."""
    from xagents_amd._lib import call, load, stream
    rng = np.random.default_rng(rows + F)
    P = (W - k) // s + 1
    if u8:
        xh = rng.integers(0, 256, size=(rows, W, C), dtype=np.uint8)
        x64 = (xh.astype(np.float32) / np.float32(255.0)).astype(np.float64)
    else:
        xh = rng.normal(size=(rows, W, C)).astype(np.float32)
        x64 = xh.astype(np.float64)
    dy = rng.normal(size=(rows, P, F)).astype(np.float32)
    idx = np.arange(P)[:, None] * s + np.arange(k)[None, :]
    cols = x64[:, idx, :].reshape(rows * P, k * C)
    ref_w = cols.T @ dy.reshape(rows * P, F).astype(np.float64)
    ref_b = dy.astype(np.float64).sum((0, 1))
    n_ws = int(load().xa_conv1d_wgrad_workspace_floats(k, C, F))
    assert n_ws > 0
    ws = torch.empty(n_ws, device=device)
    tx, tdy = torch.from_numpy(xh).to(device), torch.from_numpy(dy).to(device)
    w0 = rng.normal(size=(k * C, F)).astype(np.float32)
    b0 = rng.normal(size=F).astype(np.float32)
    for acc in (0, 1):
        dw, db = torch.from_numpy(w0.copy()).to(device), torch.from_numpy(b0.copy()).to(device)
        call('xa_conv1d_wgrad', tx.data_ptr(), int(u8), tdy.data_ptr(), rows, W, C, P, k, s, F,
             dw.data_ptr(), db.data_ptr(), acc, ws.data_ptr(), n_ws, stream())
        torch.cuda.synchronize()
        _close(dw.cpu().numpy(), ref_w + (w0 if acc else 0))
        _close(db.cpu().numpy(), ref_b + (b0 if acc else 0))


@pytest.mark.parametrize('B,half', [(64, False), (64, True), (4, True)])
def test_layer_executor_cnn_backward_on_leading_rows(device, B, half):
    """The DQN learner's pattern (dqn/agent.py: one forward over [s; s'] of 2B rows, the
    backward over the first B): per-tensor norm-relative error vs float64."""
    import sys
    sys.path.insert(0, str(ROOT / 'oracle'))
    import nets_f64 as O
    from xagents_amd.layers import LayerExecutor
    model = _model(ROOT / 'xagents_amd' / 'dqn/models/cnn.cfg', [6], (84, 84, 1), device)
    rng = np.random.default_rng(5)
    R = 2 * B if half else B
    x = rng.integers(0, 256, size=(R, 84, 84, 1), dtype=np.uint8)
    ex = LayerExecutor(model, R)
    ex.forward(torch.from_numpy(x).to(device))
    dq = np.zeros((B, 6), np.float32)
    dq[np.arange(B), rng.integers(0, 6, size=B)] = rng.normal(size=B).astype(np.float32)
    grad = torch.zeros(model.n_params, device=device)
    ex.backward([torch.from_numpy(dq).to(device)], grad, batch=B)
    theta = model.theta.cpu().numpy()
    x64, ref_outs = O.forward(model.layers, theta, x[:B], (84, 84, 1))
    dev = {i: ex.outs[i][:B].cpu().numpy() for i, l in enumerate(model.layers)
           if l.kind != 'flatten'}
    ref_outs, flips = O.adopt_gates(model.layers, ref_outs, dev)
    S = np.zeros(model.n_params)
    dl = {}
    ref_g = O.backward(model.layers, theta, x64, ref_outs, {model.outputs[0]: dq}, abs_terms=S,
                       d_layers=dl)
    dz_msgs = []
    # the fused conv-stack backward keeps dZ1 / dZ2 in LDS: douts[0..1] are never written
    fused_stack = ex._stack_bwd_ok()
    for i, l in enumerate(model.layers):
        if l.kind == 'flatten' or i not in dl or ex.douts[i] is None or i in model.outputs:
            continue
        if fused_stack and i < 2:
            continue
        want = dl[i] * (ref_outs[i] > 0)
        got = ex.douts[i][:B].cpu().numpy().reshape(want.shape)
        dz_msgs.append(f'dz[{i}] {_rel_err(got, want):.2e} worst@'
                       f'{np.unravel_index(np.argmax(np.abs(got - want)), want.shape)}')
    sls, _ = O.param_slices(model.layers)
    g = grad.cpu().numpy().astype(np.float64)
    msgs, worst = [], 0.0
    for sl in sls:
        for off, s in sl or ():
            n = int(np.prod(s))
            d = np.linalg.norm(g[off:off + n] - ref_g[off:off + n])
            r = d / np.linalg.norm(ref_g[off:off + n])
            worst = max(worst, r)
            msgs.append(f'{s}: {r:.2e} (|S|/|g| {np.linalg.norm(S[off:off + n]) / np.linalg.norm(ref_g[off:off + n]):.1f})')
    assert worst < 1e-4, '; '.join(msgs + dz_msgs + [f'{flips} gate flips'])


def _rel_err(got, want):
    return float(np.linalg.norm(np.asarray(got, np.float64) - want) / np.linalg.norm(want))


@pytest.mark.parametrize('B,u8', [(1, True), (5, True), (37, False), (32, True), (64, True),
                                  (128, True)])
def test_conv_stack_fused_forward(device, B, u8, monkeypatch):
    """xa_conv_stack_fwd (the NatureCNN Conv1D stack in one launch) against the per-layer
    GEMM path and the f64 restatement: every hidden activation, f32 and uint8 frames, row
    shares that end in partial chunks of 16 frame rows (B = 1: one row per workgroup; 5, 37;
    32: 10-11 rows per workgroup; 64: 16 + 5; 128: 16 + 16 + 10); keep_hidden=False leaves the
    features bit-identical."""
    import sys
    sys.path.insert(0, str(ROOT / 'oracle'))
    import nets_f64 as O
    from xagents_amd.layers import LayerExecutor
    model = _model(ROOT / 'xagents_amd' / 'dqn/models/cnn.cfg', [6], (84, 84, 1), device)
    rng = np.random.default_rng(B)
    x = (rng.integers(0, 256, size=(B, 84, 84, 1), dtype=np.uint8) if u8 else
         rng.random(size=(B, 84, 84, 1)).astype(np.float32))
    xt = torch.from_numpy(x).to(device)
    monkeypatch.setenv('XA_CONV_STACK', '0')
    ex0 = LayerExecutor(model, B)
    monkeypatch.setenv('XA_CONV_STACK', '1')
    ex1, ex2 = LayerExecutor(model, B), LayerExecutor(model, B)
    assert not ex0.stack and ex1.stack and ex2.stack
    ex2.keep_hidden = False
    o0, o1, o2 = ex0.forward(xt), ex1.forward(xt), ex2.forward(xt)
    _, ref = O.forward(model.layers, model.theta.cpu().numpy(), x, (84, 84, 1))
    for i in range(3):
        _close(ex1.outs[i].cpu().numpy(), ex0.outs[i].cpu().numpy(), rtol=1e-5)
        _close(ex1.outs[i].cpu().numpy(), ref[i])
    assert torch.equal(ex2.outs[2], ex1.outs[2])
    for a, b, c in zip(o0, o1, o2):
        _close(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-5)
        assert torch.equal(b, c)


@pytest.mark.parametrize('B,Bb,u8,acc', [(2, 2, True, False), (5, 3, True, True),
                                         (37, 37, False, False), (64, 64, True, False),
                                         (128, 128, True, False)])
def test_conv_stack_fused_backward(device, B, Bb, u8, acc, monkeypatch):
    """xa_conv_stack_bwd (the stack's weight / bias gradients in one launch + a fixed-order
    reduce) against the per-layer GEMM backward on the same forward: all six parameter
    tensors at 1e-5 of their scale, a leading-rows batch (Bb < B), accumulate=True, ragged
    last groups; the dense layers' gradients are untouched by the switch (bitwise)."""
    from xagents_amd.layers import LayerExecutor
    model = _model(ROOT / 'xagents_amd' / 'dqn/models/cnn.cfg', [6], (84, 84, 1), device)
    rng = np.random.default_rng(100 + B)
    x = (rng.integers(0, 256, size=(B, 84, 84, 1), dtype=np.uint8) if u8 else
         rng.random(size=(B, 84, 84, 1)).astype(np.float32))
    xt = torch.from_numpy(x).to(device)
    ex = LayerExecutor(model, B)
    assert ex.stack and ex._stack_bwd_ok()
    outs = ex.forward(xt)
    d = torch.from_numpy(rng.normal(size=(Bb, 6)).astype(np.float32)).to(device)
    base = torch.from_numpy(rng.normal(size=model.n_params).astype(np.float32)).to(device)
    grads = []
    for flag in ('0', '1'):
        monkeypatch.setenv('XA_CONV_STACK_BWD', flag)
        g = base.clone() if acc else torch.zeros_like(base)
        ex.backward([d], g, batch=Bb, accumulate=acc)
        grads.append(g.cpu().numpy())
    ref, got = grads
    n_conv = ex.offsets[2][1] + model.layers[2].filters
    for i in range(3):
        (w0, b0), l = ex.offsets[i], model.layers[i]
        for lo, hi in ((w0, b0), (b0, b0 + l.filters)):
            _close(got[lo:hi], ref[lo:hi], rtol=1e-5)
    assert np.array_equal(got[n_conv:], ref[n_conv:])
