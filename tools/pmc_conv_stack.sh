# PMC passes (two, each within the per-block counter limits) on the fused conv-stack
# backward at 1024 frames; run on the GPU box: bash tools/pmc_conv_stack.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $R/gpurun_out/r05zz_pmc1 -o run --output-format csv -- python $R/tools/conv_stack_bwd_once.py > $R/gpurun_out/r05zz_pmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $R/gpurun_out/r05zz_pmc2 -o run --output-format csv -- python $R/tools/conv_stack_bwd_once.py > $R/gpurun_out/r05zz_pmc2.log 2>&1 || exit $?
