#!/bin/bash
# round 2: two-level (XCD-local) exchange -- update tests, stamps, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02f}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ppo_update.py tests/test_gpu_agent.py > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 200 python tools/diag_ppo_update.py --no-build > gpurun_out/${T}_diag.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 2 \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
