set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 150 python tools/adam_stream_probe.py 30 > gpurun_out/r06zj_adam_probe.txt 2>&1
cat gpurun_out/r06zj_adam_probe.txt
B="python bench.py --config c3 --steps 40 --warmup 5 --cpu-baseline-seconds 0"
for i in 1 2; do
  XA_DQN_STAGE_EARLY=0 timeout -k 10 200 $B > gpurun_out/r06zj_c3_off$i.json 2> gpurun_out/r06zj_c3_off$i.err
  timeout -k 10 200 $B > gpurun_out/r06zj_c3_on$i.json 2> gpurun_out/r06zj_c3_on$i.err
done
python tools/bench_brief.py gpurun_out/r06zj_c3_*.json || true
timeout -k 10 400 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_gpu_dqn.py tests/test_gpu_configs.py::test_c3_dqn_32_envs_rb1_1m_batch_64 > gpurun_out/r06zj_dqn.log 2>&1
tail -3 gpurun_out/r06zj_dqn.log
