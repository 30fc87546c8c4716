#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/ab_bench$i.json 2>/dev/null || exit 3
done
