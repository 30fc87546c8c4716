set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_cnn_onpolicy.py tests/test_gpu_dqn.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_layers.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_layers.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpurun_prof_c4.sh
