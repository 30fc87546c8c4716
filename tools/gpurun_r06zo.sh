set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r06zo
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_kernels.py tests/test_gpu_ppo_update.py tests/test_gpu_agent.py tests/test_gpu_walker.py > gpurun_out/${T}_roll.log 2>&1 || { tail -40 gpurun_out/${T}_roll.log; exit 1; }
tail -2 gpurun_out/${T}_roll.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
TAG=$T bash tools/gpu_steps.sh prof
B="python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-secondary"
timeout -k 10 200 $B > gpurun_out/${T}_b1.json 2> gpurun_out/${T}_b1.err
timeout -k 10 200 $B > gpurun_out/${T}_b2.json 2> gpurun_out/${T}_b2.err
python tools/bench_brief.py gpurun_out/${T}_b*.json gpurun_out/${T}_prof_bench.json || true
grep -E "replay_rollout|mlp_rollout_kernel" gpurun_out/${T}_prof/run_kernel_stats.csv | cut -c1-160
