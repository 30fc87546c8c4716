#!/bin/bash
# quick GPU loop: kernel tests + bench + kernel-trace summary (each step time-limited)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${QUICK_TESTS:-tests/test_gpu_kernels.py} -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 2; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/bench_quick.log 2>&1 || exit 3
tail -1 gpurun_out/bench_quick.log | cut -c1-900
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profq -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/profq.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT && python - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/profq/run_kernel_stats.csv')))
for r in rows[:12]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
