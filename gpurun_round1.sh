#!/bin/bash
# one GPU call: tests -> smoke -> bench -> rocprofv3 kernel trace (stop on any fault)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/rocm_smi.txt 2>&1 || true
timeout -k 10 420 python -m pytest tests -q -m gpu -p no:cacheprovider 2>&1 | tee gpurun_out/pytest_gpu.log
rc=${PIPESTATUS[0]}
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | tee gpurun_out/bench.log || exit 4
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || exit 5
echo done
