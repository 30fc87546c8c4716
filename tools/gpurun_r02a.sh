#!/bin/bash
# round 2: persistent PPO update -- GPU tests of the update path, then a short bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_ppo_update.py tests/test_gpu_agent.py > gpurun_out/r02a_pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 5 \
  > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err
