#!/bin/bash
# round 2: update stamp breakdown, per-shape kernel-trace summaries and PMC traffic passes
# (16 envs = the metric's workload, 256 envs = C2). One counter per PMC pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
T=${TAG:-r02n}
cd $R && timeout -k 10 200 python tools/diag_ppo_update.py --no-build > gpurun_out/${T}_diag.txt 2>&1 || exit 3
cd /tmp
for n in 16 256; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof_n$n -o run \
    --output-format csv -- python $R/bench.py --n-envs $n --no-c2 --steps 10 --warmup 3 \
    --cpu-baseline-seconds 0 > $R/gpurun_out/${T}_prof_n$n.log 2>&1 || exit 5
done
for n in 16 256; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${T}_n${n}_$c -o run \
      --output-format csv -- python $R/bench.py --n-envs $n --no-c2 --steps 2 --warmup 1 \
      --cpu-baseline-seconds 0 --no-graph > $R/gpurun_out/pmc_${T}_n${n}_$c.log 2>&1 || exit 7
  done
done
echo done
