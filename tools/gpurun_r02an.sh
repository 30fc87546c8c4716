#!/bin/bash
# validation of the round's tree: every -m gpu test, smoke, bench line (+ CPU baseline),
# kernel-trace summary, per-shape PMC traffic passes, C3 secondary line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r02an}
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err &&
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run --output-format csv \
  -- python $R/bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $R/gpurun_out/${T}_prof_bench.json 2>&1) &&
TAG=${T} bash tools/gpurun_pmc_shapes.sh > gpurun_out/${T}_pmc.log 2>&1 &&
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0 \
  > gpurun_out/${T}_bench_c3.json 2> gpurun_out/${T}_bench_c3.err &&
exit $rc
