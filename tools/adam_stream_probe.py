"""(diagnostic) C3's dense weight-gradient GEMM with Adam in its epilogue (xa_gemm_adam,
37633 x 512 x 64) against a plain streaming Adam over the same parameters (xa_clip_adam, no
clip) and a float4 copy of the same bytes: HIP-event time and achieved GB/s of each, to see
how far the fused launch is from the streaming rate the part reaches.

    python tools/adam_stream_probe.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xagents_amd import kernels  # noqa: E402
from xagents_amd.layers import adam_apply, gemm_adam  # noqa: E402


class _Opt:
    learning_rate, beta_1, beta_2, epsilon = 1e-4, 0.9, 0.999, 1e-7


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2], ts[0]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = 'cuda'
    n_in, n_out, B = 37632, 512, 64
    P = (n_in + 1) * n_out
    g = torch.Generator(device='cpu').manual_seed(5)
    src = torch.randn(B, n_in, generator=g).to(dev)
    d = torch.randn(B, n_out, generator=g).to(dev)
    th = torch.randn(P, generator=g).to(dev)
    m = torch.zeros(P, device=dev)
    v = torch.zeros(P, device=dev)
    grad = torch.randn(P, generator=g).to(dev)
    step = torch.ones(1, dtype=torch.int32, device=dev)
    ad = adam_apply(th, m, v, step, _Opt, 0)

    def fused():
        gemm_adam(n_in + 1, n_out, B, src.data_ptr(), d.data_ptr(), None, ad, a_m=(1, 1, 0),
                  a_k=(1, n_in, 0), b_ks=n_out, b_ns=1, ldc=n_out, a_ones_row=True)

    def plain():
        kernels.clip_adam(th, m, v, grad, step, 1e-4, 0.9, 0.999, 1e-7, clip_norm=0.0)

    dst = torch.empty(3 * P, device=dev)
    srcc = torch.randn(3 * P, generator=g).to(dev)

    def copy():
        dst.copy_(srcc)

    rows = [('xa_gemm_adam 37633x512x64', fused, 24 * P + 4 * B * (n_in + n_out)),
            ('xa_clip_adam (no clip)', plain, 28 * P),
            ('copy of theta/m/v bytes', copy, 24 * P)]
    for name, fn, nbytes in rows:
        med, best = timed(fn, reps)
        print(f'{name:30s} median {med:7.1f} us  best {best:7.1f} us  '
              f'{nbytes / med / 1e3:7.1f} GB/s (median)  {nbytes / 1e6:.1f} MB', flush=True)


if __name__ == '__main__':
    main()
