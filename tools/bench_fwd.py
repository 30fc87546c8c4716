"""Timing of xa_gemm on the NatureCNN dense layer's FORWARD shape (M x 512 x 37632, A
row-major, W [K][N], bias + ReLU, xa_gemm_splits' split count) at the acting / learner
batches: the split-K forward kernel vs the generic tile kernels (force_small = 1); us per
launch including the split reduce (HIP events, 50 launches).
usage: python tools/bench_fwd.py [M ...]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd import _lib
    from xagents_amd._lib import XA_ACT_RELU
    from xagents_amd.layers import gemm
    import os
    # XA_LIB: a variant build (tools/build_variant.py) instead of the product
    lib = _lib.load(os.environ['XA_LIB']) if os.environ.get('XA_LIB') else _lib.load()
    _lib._lib = lib
    dev = torch.device('cuda')
    N, K = 512, 37632
    for M in [int(a) for a in sys.argv[1:]] or [16, 32, 64]:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) * 0.01
        bias = torch.randn(N, device=dev)
        c = torch.empty(M, N, device=dev)
        s = lib.xa_gemm_splits(M, N, K)
        ws = torch.empty(max(s, 1) * M * N + 1, device=dev)
        for label, force in (('split-K fwd', 4), ('default', 0)):
            def run():
                gemm(M, N, K, a.data_ptr(), w.data_ptr(), c.data_ptr(), a_m=(1, K, 0), b_ks=N,
                     b_ns=1, ldc=N, bias=bias.data_ptr(), act=XA_ACT_RELU, workspace=ws,
                     splits=s, force_small=force)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            reps = 50
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            gbs = (4.0 * (K * N + M * K)) / (us * 1e-6) / 1e9
            print(f'dense fwd M={M:3d} splits={s:3d} {label:11s}: {us:8.2f} us  {tf:6.2f} TF/s  '
                  f'{gbs:7.1f} GB/s of W + A', flush=True)


if __name__ == '__main__':
    main()
