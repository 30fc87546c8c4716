set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_td3.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_td3.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_td3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 100 --warmup 10 > gpurun_out/bench_c5.log 2>&1 && tail -1 gpurun_out/bench_c5.log | cut -c 1-200,600-900
