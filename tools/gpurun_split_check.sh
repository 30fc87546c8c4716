#!/bin/bash
# after a GEMM dispatch change: GPU tests, split sweep, CNN config lines (no CPU baselines)
set -u
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 240 python tools/gemm_split_sweep.py > gpurun_out/split_sweep.txt 2>&1 &&
timeout -k 10 120 python tools/acer_breakdown.py > gpurun_out/acer_breakdown.txt 2>&1 && cat gpurun_out/acer_breakdown.txt &&
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/bench_c3.log 2>&1 && tail -1 gpurun_out/bench_c3.log &&
timeout -k 10 300 python bench.py --config acer --steps 20 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/bench_acer.log 2>&1 && tail -1 gpurun_out/bench_acer.log &&
timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/bench_c4.log 2>&1 && tail -1 gpurun_out/bench_c4.log
