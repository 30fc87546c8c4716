set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trpo.py tests/test_gpu_layers.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_trpo.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_trpo.log; exit $rc
