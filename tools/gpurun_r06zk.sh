set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r06zk
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_layers.py -k "gemm_adam or ones_row" > gpurun_out/${T}_layers.log 2>&1 || { tail -30 gpurun_out/${T}_layers.log; exit 1; }
tail -2 gpurun_out/${T}_layers.log
XA_GEMM_ADAM_PERSIST=0 timeout -k 10 200 $PYT tests/test_gpu_layers.py -k "gemm_adam" > gpurun_out/${T}_layers_off.log 2>&1
tail -2 gpurun_out/${T}_layers_off.log
for i in 1 2; do
  XA_GEMM_ADAM_PERSIST=0 timeout -k 10 150 python tools/adam_stream_probe.py 30 > gpurun_out/${T}_probe_off$i.txt 2>&1
  timeout -k 10 150 python tools/adam_stream_probe.py 30 > gpurun_out/${T}_probe_on$i.txt 2>&1
done
grep -h gemm_adam gpurun_out/${T}_probe_*.txt
timeout -k 10 400 $PYT tests/test_gpu_dqn.py tests/test_gpu_configs.py::test_c3_dqn_32_envs_rb1_1m_batch_64 > gpurun_out/${T}_dqn.log 2>&1
tail -2 gpurun_out/${T}_dqn.log
B="python bench.py --config c3 --steps 40 --warmup 5 --cpu-baseline-seconds 0"
for i in 1 2; do
  XA_GEMM_ADAM_PERSIST=0 timeout -k 10 200 $B > gpurun_out/${T}_c3_off$i.json 2> gpurun_out/${T}_c3_off$i.err
  timeout -k 10 200 $B > gpurun_out/${T}_c3_on$i.json 2> gpurun_out/${T}_c3_on$i.err
done
python tools/bench_brief.py gpurun_out/${T}_c3_*.json || true
