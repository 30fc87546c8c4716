#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02x}
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_configs.py > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 200 python tools/diag_ppo_update.py --no-build 16 256 > gpurun_out/${T}_diag.txt 2>&1
