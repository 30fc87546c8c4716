#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ppo_update.py tests/test_gpu_agent.py > gpurun_out/r02q_pytest.log 2>&1 &&
timeout -k 10 200 python tools/diag_graph_fast.py > gpurun_out/r02q_graph_fast.txt 2>&1
