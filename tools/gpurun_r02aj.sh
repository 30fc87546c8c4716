#!/bin/bash
# PMC passes on the dense input-gradient GEMM: M = 64 (small-M kernel) and M = 4096 (tile kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/pmc_aj
export TMPDIR=/tmp
cd /tmp
for B in 64 4096; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc_aj/p1_$B -o run --output-format csv -- python $R/tools/gemm_one.py 'dense dX' 10 $B > $R/gpurun_out/pmc_aj/p1_$B.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAVES -d $R/gpurun_out/pmc_aj/p2_$B -o run --output-format csv -- python $R/tools/gemm_one.py 'dense dX' 10 $B > $R/gpurun_out/pmc_aj/p2_$B.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_aj/p3_$B -o run --output-format csv -- python $R/tools/gemm_one.py 'dense dX' 10 $B > $R/gpurun_out/pmc_aj/p3_$B.log 2>&1 || exit 5
done
echo ok
