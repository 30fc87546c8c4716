#!/bin/bash
# A/B: episode-statistics copy on the launch stream (one graph per step) vs on a side stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/r02ao_main$i.json 2>/dev/null || exit 3
XA_STATS_SIDE_STREAM=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/r02ao_side$i.json 2>/dev/null || exit 4
done
