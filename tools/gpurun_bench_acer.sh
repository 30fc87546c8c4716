#!/bin/bash
# ACER bench line + kernel trace summary
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config acer --steps 20 --warmup 5 > gpurun_out/bench_acer.log 2>&1 || exit 4
tail -1 gpurun_out/bench_acer.log
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_acer -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config acer --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_acer.log 2>&1 || exit 5
echo done
