set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r06zp
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_layers.py -k "gemm_adam" > gpurun_out/${T}_adx.log 2>&1 || { tail -40 gpurun_out/${T}_adx.log; exit 1; }
tail -2 gpurun_out/${T}_adx.log
timeout -k 10 500 $PYT tests/test_gpu_dqn.py tests/test_gpu_configs.py tests/test_gpu_layers.py > gpurun_out/${T}_dqn.log 2>&1 || { tail -40 gpurun_out/${T}_dqn.log; exit 1; }
tail -2 gpurun_out/${T}_dqn.log
B="python bench.py --config c3 --steps 40 --warmup 5 --cpu-baseline-seconds 0"
for i in 1 2; do
  XA_FUSED_DX=0 timeout -k 10 200 $B > gpurun_out/${T}_c3_off$i.json 2> gpurun_out/${T}_c3_off$i.err
  timeout -k 10 200 $B > gpurun_out/${T}_c3_on$i.json 2> gpurun_out/${T}_c3_on$i.err
done
python tools/bench_brief.py gpurun_out/${T}_c3_*.json || true
TAG=$T bash tools/gpu_steps.sh profc3
cat gpurun_out/${T}_profc3_timeline.txt
