set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config trpo --steps 5 --warmup 2 > gpurun_out/bench_trpo.log 2>&1 && tail -1 gpurun_out/bench_trpo.log &&
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_trpo -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config trpo --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_trpo.log 2>&1
