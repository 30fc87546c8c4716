set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc/a1 -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --cpu-baseline-seconds 0 --no-graph > $R/gpurun_out/pmc/a1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAVES -d $R/gpurun_out/pmc/a2 -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --cpu-baseline-seconds 0 --no-graph > $R/gpurun_out/pmc/a2.log 2>&1
echo rc=$?
