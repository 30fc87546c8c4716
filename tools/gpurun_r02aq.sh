#!/bin/bash
# step-per-lane replay rollout: rollout kernel tests first, then every -m gpu test
# then two bench lines (16-env headline + C2) (no CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02aq}
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_agent.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest0.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 \
  > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || exit 5
done
