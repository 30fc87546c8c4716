#!/bin/bash
# per-shape kernel-trace summaries and PMC traffic passes (one counter per pass) of the
# bench's 16-env (metric) and 256-env (C2) workloads
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
T=${TAG:-r02y}
cd /tmp
for n in 16 256; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof_n$n -o run \
    --output-format csv -- python $R/bench.py --n-envs $n --no-c2 --steps 20 --warmup 5 \
    --cpu-baseline-seconds 0 --no-secondary > $R/gpurun_out/${T}_prof_n$n.log 2>&1 || exit 5
done
for n in 16 256; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${T}_n${n}_$c -o run \
      --output-format csv -- python $R/bench.py --n-envs $n --no-c2 --steps 2 --warmup 1 \
      --cpu-baseline-seconds 0 --no-graph --no-secondary > $R/gpurun_out/pmc_${T}_n${n}_$c.log 2>&1 || exit 7
  done
done
echo done
