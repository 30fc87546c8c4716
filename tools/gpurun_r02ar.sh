#!/bin/bash
# rollout change: kernel / agent / play tests, then two bench lines (16-env headline + C2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02ar}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_agent.py \
  tests/test_gpu_play.py tests/test_gpu_hooks.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 \
  > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || exit 5
done
