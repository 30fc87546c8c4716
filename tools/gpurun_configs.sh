#!/bin/bash
# secondary-config benches (C3 DQN, C4 PPO-CNN, C5 TD3, TRPO, ACER), each under its own time limit
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config c3 --steps 30 --warmup 5 > gpurun_out/bench_c3.log 2>&1 && tail -1 gpurun_out/bench_c3.log &&
timeout -k 10 300 python bench.py --config c5 --steps 100 --warmup 10 > gpurun_out/bench_c5.log 2>&1 && tail -1 gpurun_out/bench_c5.log &&
timeout -k 10 500 python bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/bench_c4.log 2>&1 && tail -1 gpurun_out/bench_c4.log &&
timeout -k 10 300 python bench.py --config trpo --steps 5 --warmup 2 > gpurun_out/bench_trpo.log 2>&1 && tail -1 gpurun_out/bench_trpo.log &&
timeout -k 10 300 python bench.py --config acer --steps 20 --warmup 5 > gpurun_out/bench_acer.log 2>&1 && tail -1 gpurun_out/bench_acer.log
