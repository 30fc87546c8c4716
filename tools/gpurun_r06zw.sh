set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r06zw
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_layers.py tests/test_gpu_dqn.py tests/test_gpu_configs.py tests/test_gpu_cnn_onpolicy.py > gpurun_out/${T}_cnn.log 2>&1 || { tail -40 gpurun_out/${T}_cnn.log; exit 1; }
tail -2 gpurun_out/${T}_cnn.log
TAG=$T bash tools/gpu_steps.sh profc3 profc4
cat gpurun_out/${T}_profc3_timeline.txt | grep -E "span|bwd"
grep -E "conv_stack" gpurun_out/${T}_profc4_shapes.txt
