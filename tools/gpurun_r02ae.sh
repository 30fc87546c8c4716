#!/bin/bash
# walker stand-in + play + executor-path regressions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_walker.py tests/test_gpu_play.py tests/test_gpu_distributions.py tests/test_gpu_td3.py \
  tests/test_gpu_atari.py > gpurun_out/r02ae_pytest.log 2>&1
