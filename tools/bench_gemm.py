"""Per-shape timing of xa_gemm (small 64x64 kernel vs the 32x32-MFMA tile kernel) on
the CNN's forward / backward GEMM shapes (NatureCNN Conv1D cfg) at batch B."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def shapes(B):
    r = B * 84
    # name, M, N, K, a_m, a_k, b_ks, b_ns, u8
    return [
        ('conv1 fwd', r * 20, 32, 8, (20, 84, 4), (1, 1, 0), 32, 1, True),
        ('conv2 fwd', r * 9, 64, 128, (9, 640, 64), (1, 1, 0), 64, 1, False),
        ('conv3 fwd', r * 7, 64, 192, (7, 576, 64), (1, 1, 0), 64, 1, False),
        ('dense fwd', B, 512, 37632, (1, 37632, 0), (1, 1, 0), 512, 1, False),
        ('dense dW', 37632, 512, B, (1, 1, 0), (1, 37632, 0), 512, 1, False),
        ('dense dX', B, 37632, 512, (1, 512, 0), (1, 1, 0), 1, 512, False),
        ('conv3 dW', 192, 64, r * 7, (1, 1, 0), (7, 576, 64), 64, 1, False),
        ('conv3 dcol', r * 7, 192, 64, (1, 64, 0), (1, 1, 0), 1, 64, False),
        ('conv2 dW', 128, 64, r * 9, (1, 1, 0), (9, 640, 64), 64, 1, False),
        ('conv2 dcol', r * 9, 128, 64, (1, 64, 0), (1, 1, 0), 1, 64, False),
        ('conv1 dW', 8, 32, r * 20, (1, 1, 0), (20, 84, 4), 32, 1, True),
        ('bias conv2', 1, 64, r * 9, (1, 0, 0), (1, 0, 0), 64, 1, False),
    ]


def main():
    from xagents_amd import _lib
    from xagents_amd.layers import gemm
    lib = _lib.load()
    dev = torch.device('cuda')
    for B in [int(b) for b in (sys.argv[1:] or ['64', '4096'])]:
        big = torch.randn(B * 84 * 20 * 192, device=dev)  # covers every operand
        u8 = torch.randint(0, 256, (B * 84 * 84,), dtype=torch.uint8, device=dev)
        w = torch.randn(37632 * 512, device=dev)
        out = torch.empty(max(B * 84 * 20 * 192, 37632 * 512), device=dev)
        for name, M, N, K, am, ak, bks, bns, is_u8 in shapes(B):
            s = lib.xa_gemm_splits(M, N, K)
            ws = torch.empty(max(s * M * N, 1), device=dev)
            a = u8 if is_u8 else big
            bsrc = w if name.startswith('dense') or 'fwd' in name or 'dcol' in name else big
            res = []
            for small in (True, False):
                fn = lambda: gemm(M, N, K, None if name.startswith('bias') else a.data_ptr(),  # noqa: E731
                                  bsrc.data_ptr(), out.data_ptr(), a_u8=is_u8, a_m=am, a_k=ak,
                                  b_ks=bks, b_ns=bns, ldc=N, workspace=ws, force_small=small)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                n = 10
                e0.record()
                for _ in range(n):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / n * 1e3
                res.append(us)
            fl = 2.0 * M * N * K
            print(f'B={B:5d} {name:11s} M={M:9d} N={N:6d} K={K:9d} splits={s:5d}  '
                  f'small {res[0]:9.1f} us ({fl / res[0] / 1e6:6.1f} TF/s)  '
                  f'tile {res[1]:9.1f} us ({fl / res[1] / 1e6:6.1f} TF/s)', flush=True)
        del big, u8, w, out


if __name__ == '__main__':
    main()
