set -u
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/b_pro.log 2>&1 && tail -1 gpurun_out/b_pro.log | cut -c1-400 &&
XA_PPO_OPT=kernel timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/b_ker.log 2>&1 && tail -1 gpurun_out/b_ker.log | cut -c1-400 &&
XA_PPO_OPT=kernel timeout -k 10 120 python -u -m pytest tests/test_gpu_agent.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/p_ker.log 2>&1; tail -2 gpurun_out/p_ker.log
