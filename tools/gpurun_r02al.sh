#!/bin/bash
# data-parallel persistent update: DP / peer tests, update tests, 2-rank shared-GPU bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02al}
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_dp.py tests/test_gpu_peer.py tests/test_gpu_ppo_update.py > gpurun_out/${T}_pytest.log 2>&1 &&
XA_BENCH_SHARED_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr=127.0.0.1 --master-port=29622 bench.py --gpus 2 --steps 10 --warmup 3 --cpu-baseline-seconds 0 \
  > gpurun_out/${T}_shared2.log 2>&1
