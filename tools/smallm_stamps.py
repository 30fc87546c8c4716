"""Per-round shader-clock stamps of the small-M dense dX kernel (diagnostic build
XA_SMALLM_DIAG=3: tools/build_variant.py sdiag3 -DXA_SMALLM_DIAG=3 --src gemm): runs
dX = dY W^T (M x 37632 x 512, ReLU gate) and prints, averaged over the waves, the cycles of the
A prologue and of every round's chunk loop and reduce / epilogue, plus the spread of the
waves' start and end stamps.
usage: XA_LIB=tools/diag_lib/libxa_sdiag3.so python tools/smallm_stamps.py [M ...]"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd import _lib
    from xagents_amd.layers import gemm
    lib = _lib.load(os.environ['XA_LIB'])
    _lib._lib = lib
    dev = torch.device('cuda')
    N, K = 37632, 512
    for M in [int(a) for a in sys.argv[1:]] or [64]:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.01
        gate = torch.randn(M, N, device=dev)
        c = torch.empty(M, N, device=dev)
        ws = torch.zeros(2 * M * N + 1, device=dev)

        def run():
            gemm(M, N, K, a.data_ptr(), w.data_ptr(), c.data_ptr(), a_m=(1, K, 0), b_ks=1,
                 b_ns=K, ldc=N, gate=gate.data_ptr(), ld_gate=N, workspace=ws, splits=2)
        for _ in range(20):
            run()
        torch.cuda.synchronize()
        ws.zero_()
        run()
        torch.cuda.synchronize()
        t = ws[:256 * 8 * 16 * 2].view(torch.int64).cpu().numpy().reshape(256, 8, 16).astype(np.int64)
        live = t[:, :, 0] > 0
        t0 = t[:, :, 0][live].min()
        print(f'M={M}: {live.sum()} waves stamped; kernel span {t[:, :, 1:].max() - t0} cycles '
              f'(start spread {t[:, :, 0][live].max() - t0})')
        print(f'  prologue (A into LDS + first B loads): {np.mean(t[:, :, 1] - t[:, :, 0]):.0f}')
        prev = t[:, :, 1]
        for r in range(7):
            done, end = t[:, :, 2 + 2 * r], t[:, :, 3 + 2 * r]
            if not (done > 0).any():
                break
            print(f'  round {r}: chunk loop {np.mean(done - prev):7.0f}  reduce/epilogue '
                  f'{np.mean(end - done):6.0f}  (chunk loop max {np.max(done - prev)})')
            prev = end


if __name__ == '__main__':
    main()
