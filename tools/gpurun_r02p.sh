#!/bin/bash
# round 2: graph-replay correctness of the persistent update at the bench shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r02p}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ppo_update.py -k "graph_replays or block_count or persistent_update_matches" \
  > gpurun_out/${T}_pytest.log 2>&1
