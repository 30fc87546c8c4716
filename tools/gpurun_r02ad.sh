#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_smallm.py 4 16 64 128 336 > gpurun_out/r02ad_smallm.txt 2>&1
