"""Timing of xa_gemm on the dense layer's input-gradient shape dX = dY W^T
(M x 37632 x 512, B read k-major, ReLU gate) at the batches that reach the small-M kernel
(C3 64, ACER 336) plus 128, against the generic tile kernels (force_small = 2); prints us
per launch and TFLOP/s (HIP events, 50 launches)."""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd import _lib
    from xagents_amd.layers import gemm
    # XA_LIB: a diagnostic variant library (tools/build_variant.py) instead of the product
    lib = _lib.load(os.environ['XA_LIB']) if os.environ.get('XA_LIB') else _lib.load()
    _lib._lib = lib
    dev = torch.device('cuda')
    # XA_SMALLM_K: the depth (128 / 256 / 512 reach the small-M kernel; no shipped cfg has a
    # 128-unit dense layer, ADVICE r03: measure the K = 128 sub-row padding)
    N, K = 37632, int(os.environ.get('XA_SMALLM_K', '512'))
    for M in [int(a) for a in sys.argv[1:]] or [64, 128, 336]:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.01
        gate = torch.randn(M, N, device=dev)
        c = torch.empty(M, N, device=dev)
        s = lib.xa_gemm_splits(M, N, K)
        ws = torch.empty(max(s, 1) * M * N + 1, device=dev)

        for label, force in (('small-M', 0), ('generic', 2)):
            def run():
                gemm(M, N, K, a.data_ptr(), w.data_ptr(), c.data_ptr(), a_m=(1, K, 0), b_ks=1,
                     b_ns=K, ldc=N, gate=gate.data_ptr(), ld_gate=N, workspace=ws,
                     force_small=force)
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
            print(f'dense dX M={M:4d} {label:8s}: {us:8.2f} us  {tf:7.2f} TFLOP/s  '
                  f'{tf / 157.3:.3f} of peak')


if __name__ == '__main__':
    main()
