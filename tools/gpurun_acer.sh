#!/bin/bash
# ACER GPU tests (kernel + update parity, replay train steps)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_acer.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_acer.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_acer.log
exit $rc
