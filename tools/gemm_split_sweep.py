"""Sweep the K-split count of xa_gemm on the NatureCNN dense-layer shapes at the batch
sizes of C3 (64, 128 with double DQN), ACER (336) and C4 (4096): per-launch time (HIP events,
10 launches after 3 warm-ups) for splits 1..16 next to the current xa_gemm_splits choice.
usage: python tools/gemm_split_sweep.py [B ...]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tools'))


def main():
    from bench_gemm import shapes
    from xagents_amd import _lib
    from xagents_amd.layers import gemm
    lib = _lib.load()
    dev = torch.device('cuda')
    w = torch.randn(37632 * 512, device=dev)
    for B in [int(b) for b in (sys.argv[1:] or ['64', '128', '336', '4096'])]:
        big = torch.randn(max(B * 37632, 37632 * 512), device=dev)
        out = torch.empty(max(B * 37632, 37632 * 512), device=dev)
        for name, M, N, K, am, ak, bks, bns, is_u8 in shapes(B):
            if not (name.startswith('dense') or name.startswith('conv') and 'dcol' not in name):
                continue
            cur = lib.xa_gemm_splits(M, N, K)
            ws = torch.empty(min(512 * M * N, 1 << 28), device=dev)
            row = []
            for s in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
                if (K + s - 1) // s < 16 or s * M * N > ws.numel():
                    continue
                fn = lambda: gemm(M, N, K, big.data_ptr(), w.data_ptr(), out.data_ptr(),  # noqa
                                  a_m=am, a_k=ak, b_ks=bks, b_ns=bns, ldc=N, workspace=ws,
                                  splits=s)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                row.append(f's{s}={ms * 1e3:.1f}us({2 * M * N * K / ms / 1e9:.0f}TF)')
            print(f'B={B} {name} {M}x{N}x{K} cur={cur}: ' + ' '.join(row), flush=True)


if __name__ == '__main__':
    main()
