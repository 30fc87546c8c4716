#!/bin/bash
# N > 1 rehearsal on the one-GPU box: 2 ranks share cuda:0 (gloo group), bench line with the
# peer exchange and with the process-group fallback
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export XA_BENCH_SHARED_DEVICE=1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29612 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/r02ak_shared2.log 2>&1 &&
XA_PEER_ALLREDUCE=0 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr=127.0.0.1 --master-port=29613 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-baseline-seconds 0 \
  > gpurun_out/r02ak_shared2_pg.log 2>&1
