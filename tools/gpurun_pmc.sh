#!/bin/bash
# HBM traffic per launch from PMC counters, one counter per rocprofv3 pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no trace domains).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_$c -o run --output-format csv \
    -- python $R/bench.py --steps 2 --warmup 1 --cpu-baseline-seconds 0 --no-graph \
    > $R/gpurun_out/pmc_$c.log 2>&1 || exit 7
done
echo pmc done
