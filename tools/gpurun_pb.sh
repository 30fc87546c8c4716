set -u
mkdir -p gpurun_out
for pb in 64 32 16; do
XA_REDUCE_PB=$pb timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/b_pb$pb.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/b_pb$pb.log').read().strip().splitlines()[-1]); print($pb, d['ms_per_step'], d['update_ms'], d['roofline']['launch_ms'])"
done
XA_REDUCE_PB=16 timeout -k 10 120 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/p_pb.log 2>&1; tail -1 gpurun_out/p_pb.log
