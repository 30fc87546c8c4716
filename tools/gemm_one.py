"""Run one CNN GEMM shape repeatedly (for rocprofv3 PMC passes): dense dX of the
NatureCNN dense layer at B = 4096 by default.
usage: python tools/gemm_one.py [name] [reps] [B]"""
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
    name = sys.argv[1] if len(sys.argv) > 1 else 'dense dX'
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    lib = _lib.load()
    dev = torch.device('cuda')
    (_, M, N, K, am, ak, bks, bns, is_u8), = [s for s in shapes(B) if s[0] == name]
    a = torch.randn(max(M * K, 1), device=dev)
    b = torch.randn(max(K * N, 1), device=dev)
    c = torch.empty(M * N, device=dev)
    s = lib.xa_gemm_splits(M, N, K)
    ws = torch.empty(max(s * M * N, 1), device=dev)
    for _ in range(reps):
        gemm(M, N, K, a.data_ptr(), b.data_ptr(), c.data_ptr(), a_m=am, a_k=ak, b_ks=bks,
             b_ns=bns, ldc=N, workspace=ws)
    torch.cuda.synchronize()
    print('ok', name, M, N, K)


if __name__ == '__main__':
    main()
