#!/bin/bash
# persistent-update change: update / agent tests, then the bench line (no CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02ah}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ppo_update.py tests/test_gpu_agent.py > gpurun_out/${T}_pytest.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 \
  > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || exit 5
done
