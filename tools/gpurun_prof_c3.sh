#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o run --output-format csv -- python $R/bench.py --config c3 --steps 30 --warmup 5 > $R/gpurun_out/prof_c3.log 2>&1
echo done
