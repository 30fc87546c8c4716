#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_ppo_update.py --no-build 16 256 > gpurun_out/r02r_diag.txt 2>&1
