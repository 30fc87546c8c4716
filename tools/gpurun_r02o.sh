#!/bin/bash
# round 2: persistent update duration by launch mode (graph / eager, gaps, spin)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02o}
timeout -k 10 200 python tools/diag_update_modes.py > gpurun_out/${T}_modes.txt 2>&1 &&
true || timeout -k 10 200 python tools/diag_update_modes.py --stamps > gpurun_out/${T}_modes_stamps.txt 2>&1
