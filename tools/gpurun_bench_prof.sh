#!/bin/bash
# C2 bench line + rocprofv3 kernel-trace summary of the same command
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit 4
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || exit 5
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log
