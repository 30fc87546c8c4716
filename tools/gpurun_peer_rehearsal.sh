set -u
mkdir -p gpurun_out
export PEER_TIMING=1
timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29610 tests/peer_worker.py > gpurun_out/peer_timing1.log 2>&1 || exit 2
grep "PEER" gpurun_out/peer_timing1.log
timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29611 tests/peer_worker.py > gpurun_out/peer_timing.log 2>&1 || exit 2
grep "PEER" gpurun_out/peer_timing.log
export XA_BENCH_SHARED_DEVICE=1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29612 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_shared2.log 2>&1 || exit 3
tail -1 gpurun_out/bench_shared2.log
XA_PEER_ALLREDUCE=0 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29613 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_shared2_rccl.log 2>&1 || exit 4
tail -1 gpurun_out/bench_shared2_rccl.log
