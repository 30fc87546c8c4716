#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o run --output-format csv -- python $R/bench.py --config c3 --steps 20 --warmup 3 > $R/gpurun_out/prof_c3.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run --output-format csv -- python $R/bench.py --config c4 --steps 1 --warmup 1 > $R/gpurun_out/prof_c4.log 2>&1
echo done
