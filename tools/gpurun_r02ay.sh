#!/bin/bash
# default bench line (with the CPU baseline) twice: is the C2 secondary stable?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02ay}
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
  > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || exit 5
done
