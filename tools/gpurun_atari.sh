#!/bin/bash
# Atari preprocessing parity on device, then C3 / C4 benches with and without it
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_atari.py tests/test_gpu_dqn.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_atari.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_atari.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config c3 --steps 30 --warmup 5 > gpurun_out/bench_c3.log 2>&1 && tail -1 gpurun_out/bench_c3.log &&
timeout -k 10 400 python bench.py --config c3 --preprocess --steps 30 --warmup 5 > gpurun_out/bench_c3p.log 2>&1 && tail -1 gpurun_out/bench_c3p.log &&
timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/bench_c4.log 2>&1 && tail -1 gpurun_out/bench_c4.log &&
timeout -k 10 400 python bench.py --config c4 --preprocess --steps 2 --warmup 1 > gpurun_out/bench_c4p.log 2>&1 && tail -1 gpurun_out/bench_c4p.log
