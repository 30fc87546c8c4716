#!/bin/bash
# round 2: rollout chunk pass -- rollout parity tests, agent tests, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02m}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_agent.py tests/test_gpu_hooks.py \
  > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 2 \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
