#!/bin/bash
# round 2: new GPU tests (scale-sensitive heads, DP, persistent update) + tile stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02d}
timeout -k 10 200 python tools/diag_ppo_update.py --no-build > gpurun_out/${T}_diag.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_scale.py tests/test_gpu_dp.py tests/test_gpu_ppo_update.py \
  > gpurun_out/${T}_pytest.log 2>&1
