set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trpo.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_trpo.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_trpo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config trpo --steps 5 --warmup 2 > gpurun_out/bench_trpo.log 2>&1 && tail -1 gpurun_out/bench_trpo.log | cut -c 1-80,560-700
