#!/bin/bash
# play() tests + current stamp breakdown of the persistent update at 16 envs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02ab}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_play.py > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 200 python tools/diag_ppo_update.py --no-build 16 > gpurun_out/${T}_diag.txt 2>&1
