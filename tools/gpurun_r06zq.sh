set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r06zq
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_dqn.py tests/test_gpu_configs.py tests/test_gpu_layers.py > gpurun_out/${T}_dqn.log 2>&1 || { tail -40 gpurun_out/${T}_dqn.log; exit 1; }
tail -2 gpurun_out/${T}_dqn.log
B="python bench.py --config c3 --steps 40 --warmup 5 --cpu-baseline-seconds 0"
timeout -k 10 200 $B > gpurun_out/${T}_c3_1.json 2> gpurun_out/${T}_c3_1.err
timeout -k 10 200 $B > gpurun_out/${T}_c3_2.json 2> gpurun_out/${T}_c3_2.err
python tools/bench_brief.py gpurun_out/${T}_c3_*.json || true
TAG=$T bash tools/gpu_steps.sh profc3
cat gpurun_out/${T}_profc3_timeline.txt
