#!/bin/bash
# tests/cnn_ppo_dp_worker.py at W = 2: the DP-vs-union deviation ('theta rel', which the test
# bounds) for the product library with and without the row-dot heads (XA_GEMM_FORCE=3) and
# for the variant libraries under tools/diag_lib/libxa_gold*.so, over record seeds
set -o pipefail
i=0
for SEED in 55 155 255; do
  for L in product force3 tools/diag_lib/libxa_gold*.so; do
    [ "$L" = product ] || [ "$L" = force3 ] || [ -e "$L" ] || continue
    i=$((i + 1))
    X=""; F=0
    [ "$L" = force3 ] && F=3
    [ "$L" = product ] || [ "$L" = force3 ] || X=$L
    out=$(XA_DP_SEED=$SEED XA_GEMM_FORCE=$F XA_LIB=$X HSA_ENABLE_IPC_MODE_LEGACY=0 \
      OMP_NUM_THREADS=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$((29600 + i)) \
      tests/cnn_ppo_dp_worker.py 2>&1)
    rc=$?
    echo "seed $SEED $L W=2 rc=$rc: $(echo "$out" | grep -o 'theta rel [0-9.e+-]*')"
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
  done
done
exit 0
