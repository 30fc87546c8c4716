#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run --output-format csv -- python $R/bench.py --config c4 --steps 1 --warmup 0 > $R/gpurun_out/prof_c4.log 2>&1
echo done
