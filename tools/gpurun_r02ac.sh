#!/bin/bash
# small-M GEMM: layer tests + dense dX timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02ac}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_layers.py > gpurun_out/${T}_pytest.log 2>&1 &&
timeout -k 10 120 python tools/bench_smallm.py 4 16 64 128 336 > gpurun_out/${T}_smallm.txt 2>&1
