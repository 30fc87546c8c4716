#!/bin/bash
# update-kernel iteration: update/agent tests, stamp breakdown, bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02z}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ppo_update.py tests/test_gpu_agent.py tests/test_gpu_hooks.py tests/test_gpu_checkpoint.py tests/test_gpu_dp.py > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 200 python tools/diag_ppo_update.py --no-build 16 256 > gpurun_out/${T}_diag.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
