set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_dqn.py tests/test_gpu_td3.py tests/test_gpu_cnn_onpolicy.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/bench_c4.log 2>&1 && tail -1 gpurun_out/bench_c4.log | cut -c 1-420 &&
bash tools/gpurun_prof_c4.sh
