#!/bin/bash
# tests/cnn_ppo_dp_worker.py at W = 2 / 4 with the product GEMM paths and with
# XA_GEMM_FORCE=3 (no row-dot heads): prints each run's 'theta rel' line (the DP-vs-union
# deviation the test bounds)
set -o pipefail
for F in 0 3; do
  for W in 2 4; do
    P=$((29500 + W + 10 * F))
    out=$(XA_GEMM_FORCE=$F HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1 timeout -k 10 150 \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node=$W --master-addr=127.0.0.1 \
      --master-port=$P tests/cnn_ppo_dp_worker.py 2>&1)
    rc=$?
    echo "XA_GEMM_FORCE=$F W=$W rc=$rc: $(echo "$out" | grep -o 'theta rel [0-9.e+-]*')"
    [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
  done
done
exit 0
