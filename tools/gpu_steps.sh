#!/bin/bash
# One GPU session on the gpurun box, as a list of named steps (outputs under gpurun_out/,
# prefixed with $TAG). Every GPU step has its own time limit; pytest exit 1 (test
# failures) lets the session go on, any other failure (fault, abort, time limit) ends it.
#   usage: TAG=r03a bash tools/gpu_steps.sh update bench prof ...
# steps:
#   update   tests/test_gpu_ppo_update.py
#   dp       tests/test_gpu_dp.py + tests/test_gpu_peer.py
#   gpu      the whole -m gpu suite
#   configs  tests/test_gpu_configs.py (C3 / C4 / C5 at full size)
#   variants bench A/B of tools/diag_lib/libxa_*.so (tools/build_variant.py) vs the product build
#   smoke    __graft_entry__.smoke()
#   bench    the default bench line (with the CPU baseline)
#   ab       bench lines without the CPU baseline: XCD-local vs spread persistent update
#   prof     rocprofv3 --kernel-trace --stats of the default bench (no CPU baseline)
#   pmc      FETCH_SIZE / WRITE_SIZE passes per shape (tools/gpurun_pmc_shapes.sh)
#   c3 c4 c5 acer trpo   secondary bench lines
#   pollab   persistent-update poll sleep variants: bench + C2 FETCH_SIZE
#   c2g      C2 bench lines at update grids $C2_GS (XA_PPO_MAX_BLOCKS)
#   profc3   rocprofv3 kernel trace of the C3 bench + per-(kernel, grid) summary
#   rollab   replay rollout tests, stamps (build libxa_rstamp.so first) and two bench lines
#   rstamps  per-phase stamps of the batched replay rollout (tools/rollout_stamps.py; build
#            tools/diag_lib/libxa_rstamp.so first: tools/build_variant.py rstamp -DXA_STAMPS --src mlp_rollout)
#   layers   tests/test_gpu_layers.py (GEMM paths, layer executor)
#   streamab C3 bench lines, streaming dense forward on / off, interleaved
#   stackab  C3 bench lines, fused conv-stack forward on / off, interleaved
#   bwdab    C3 / C4 bench lines, fused conv-stack backward on / off
#   cnn      CNN on-policy, ACER and Atari GPU tests
#   cstamps  per-phase stamps of the fused conv backward (tools/conv_stack_stamps.py; build
#            tools/diag_lib/libxa_cstamp.so first: tools/build_variant.py cstamp -DXA_STAMPS --src conv_stack)
#   gemm     GEMM tests, small-M timings, PMC passes on the dense dX GEMM
#   icache   instruction-cache counters of the 16-env update
#   stamps   per-phase stamp shares of the persistent update (tools/diag_ppo_update.py)
#   trace    per-block phase timeline of the persistent update (tools/trace_ppo_update.py)
#   probe    tools/probe/tile_probe (the per-step block work in isolation, old vs new tile)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
R=$PWD
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
# gpurun copies gpurun_out/ back only under 64 MiB: drop the per-dispatch kernel traces
# (the --stats summaries stay) whatever way the session ends
trap 'find gpurun_out \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete 2>/dev/null' EXIT

run_pytest() {  # name, limit, args...
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" $PYT "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  tail -3 gpurun_out/${T}_${name}.log
  case $rc in 0|1) return 0 ;; *) echo "step $name: exit $rc"; exit $rc ;; esac
}

run() {  # name, limit, command... (stdout -> .json / .log, stderr -> .err)
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_${name}.out 2> gpurun_out/${T}_${name}.err
  local rc=$?
  tail -2 gpurun_out/${T}_${name}.out
  if [ $rc -ne 0 ]; then echo "step $name: exit $rc"; tail -5 gpurun_out/${T}_${name}.err; exit $rc; fi
}

for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    update) run_pytest update 400 tests/test_gpu_ppo_update.py ;;
    dp) run_pytest dp 500 tests/test_gpu_dp.py tests/test_gpu_peer.py tests/test_gpu_rccl_capture.py ;;
    gpu) run_pytest gpu 1000 tests -m gpu ;;
    configs) run_pytest configs 400 tests/test_gpu_configs.py ;;
    td3) run_pytest td3 600 tests/test_gpu_td3.py tests/test_gpu_scale.py tests/test_gpu_configs.py::test_c5_td3_64_envs_rb2 ;;
    td3dp) run_pytest td3dp 450 tests/test_gpu_dp.py -k td3 ;;
    statab)
      # episode statistics stored by the update launch vs the xa_copy_to_host launch
      B="python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-secondary"
      run stat_on1 200 $B
      XA_STATS_IN_UPDATE=0 run stat_off1 200 $B
      run stat_on2 200 $B
      XA_STATS_IN_UPDATE=0 run stat_off2 200 $B
      python tools/bench_brief.py gpurun_out/${T}_stat_*.out ;;
    fixab)
      # the fixed-shape 16-env update kernel (BF = 3) vs the generic one, interleaved
      B="python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-secondary"
      run fix_on1 200 $B
      XA_PPO_FIXED_SHAPE=0 run fix_off1 200 $B
      run fix_on2 200 $B
      XA_PPO_FIXED_SHAPE=0 run fix_off2 200 $B
      python tools/bench_brief.py gpurun_out/${T}_fix_*.out ;;
    rollab)
      # replay rollout tests, per-phase stamps, two bench lines (the step-loop replay path it
      # replaced was A/B'd in r05ra-r05rr, profiles/r05r*_replay_rollout_ab.txt)
      run_pytest roll 200 tests/test_gpu_kernels.py -k rollout
      XA_LIB=tools/diag_lib/libxa_rstamp.so run rstamps 200 python tools/rollout_stamps.py 16 256
      B="python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-secondary"
      run roll_on1 200 $B
      run roll_on2 200 $B
      python tools/bench_brief.py gpurun_out/${T}_roll_*.out ;;
    layers) run_pytest layers 300 tests/test_gpu_layers.py ;;
    streamab)
      # the streaming few-row dense forward vs the tile kernels (XA_GEMM_STREAM=0), C3 lines
      B="python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0"
      run st_on1 300 $B
      XA_GEMM_STREAM=0 run st_off1 300 $B
      run st_on2 300 $B
      XA_GEMM_STREAM=0 run st_off2 300 $B ;;
    stackab)
      # the fused conv-stack forward vs per-layer GEMMs (XA_CONV_STACK=0), C3 lines
      B="python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0"
      run sk_on1 300 $B
      XA_CONV_STACK=0 run sk_off1 300 $B
      run sk_on2 300 $B
      XA_CONV_STACK=0 run sk_off2 300 $B ;;
    bwdab)
      # the fused conv-stack backward vs per-layer GEMMs (XA_CONV_STACK_BWD=0): C3 x2, C4 x1
      B="python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0"
      run bw_on1 300 $B
      XA_CONV_STACK_BWD=0 run bw_off1 300 $B
      run bw_on2 300 $B
      XA_CONV_STACK_BWD=0 run bw_off2 300 $B
      B4="python bench.py --config c4 --steps 3 --warmup 1 --cpu-baseline-seconds 0"
      run bw4_on 400 $B4
      XA_CONV_STACK_BWD=0 run bw4_off 400 $B4 ;;
    rstamps) XA_LIB=tools/diag_lib/libxa_rstamp.so run rstamps 200 python tools/rollout_stamps.py 16 256 ;;
    cstamps) XA_LIB=tools/diag_lib/libxa_cstamp.so run cstamps 200 python tools/conv_stack_stamps.py 64 1024 ;;
    cstampv)
      # stamp variants tools/diag_lib/libxa_<v>.so for v in $CS_VARIANTS
      for v in $CS_VARIANTS; do XA_LIB=tools/diag_lib/libxa_$v.so run cstamp_$v 200 python tools/conv_stack_stamps.py 1024; done ;;
    bwd8ab)
      # 8-wave vs 4-wave fused conv backward (XA_CONV_BWD8=0): C3 x2, C4 x1
      B="python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0"
      run b8_on1 300 $B
      XA_CONV_BWD8=0 run b8_off1 300 $B
      run b8_on2 300 $B
      XA_CONV_BWD8=0 run b8_off2 300 $B
      B4="python bench.py --config c4 --steps 3 --warmup 1 --cpu-baseline-seconds 0"
      run b84_on 400 $B4
      XA_CONV_BWD8=0 run b84_off 400 $B4 ;;
    headab)
      # DQN argmax / TD step fused into the Q head launch (default) vs separate launches
      B="python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0"
      run hd_on1 300 $B
      XA_DQN_FUSED_HEAD=0 run hd_off1 300 $B
      run hd_on2 300 $B
      XA_DQN_FUSED_HEAD=0 run hd_off2 300 $B ;;
    cnn) run_pytest cnn 600 tests/test_gpu_cnn_onpolicy.py tests/test_gpu_acer.py tests/test_gpu_atari.py ;;
    dqn) run_pytest dqn 400 tests/test_gpu_dqn.py tests/test_gpu_scale.py -k "dqn" tests/test_gpu_configs.py::test_c3_dqn_32_envs_rb1_1m_batch_64 ;;
    td3time)
      # wall time per gradient step on the product build, per-phase barrier times on the
      # trace build (tools/diag_lib/libxa_td3trace.so: tools/build_variant.py td3trace
      # -DXA_TD3_TRACE=1 --src td3_update)
      for G in ${TD3_GS:-64 128 256}; do
        XA_TD3_BLOCKS=$G run td3time_$G 120 python tools/td3_grad_steps.py 50
        XA_TD3_BLOCKS=$G XA_LIB=tools/diag_lib/libxa_td3trace.so run td3trace_$G 120 \
          python tools/td3_grad_steps.py 50
      done ;;
    c4w2)
      # W = 2 rehearsal of the C4 data-parallel bench with both ranks on the one GPU (gloo;
      # the speed means nothing, the line checks the N > 1 code path end to end)
      XA_BENCH_SHARED_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0 run c4w2 400 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py \
        --config c4 --gpus 2 --steps 2 --warmup 1 --cpu-baseline-seconds 0 ;;
    gsab)
      # train steps per graph replay (XA_GRAPH_STEPS) and events per statistics group
      # (XA_STATS_EVERY), interleaved bench lines (headline + C2, no secondaries)
      B="python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-secondary --no-dynamics"
      run gs1a 200 $B
      XA_GRAPH_STEPS=4 run gs4a 200 $B
      XA_STATS_EVERY=4 run se4a 200 $B
      run gs1b 200 $B
      XA_GRAPH_STEPS=4 run gs4b 200 $B
      XA_GRAPH_STEPS=2 run gs2b 200 $B
      python tools/bench_brief.py gpurun_out/${T}_gs*.out gpurun_out/${T}_se*.out ;;
    agent) run_pytest agent 300 tests/test_gpu_agent.py ;;
    tl16)
      # kernel trace of the 16-env headline alone: the per-step timeline (idle gaps between
      # the rollout and update launches, and between train steps)
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_tl16 \
        -o run --output-format csv -- python $R/bench.py --steps 40 --warmup 5 --no-c2 \
        --no-dynamics --no-secondary --cpu-baseline-seconds 0 > $R/gpurun_out/${T}_tl16_bench.json 2>&1) || exit $?
      python tools/step_timeline.py gpurun_out/${T}_tl16/run_kernel_trace.csv ppo_update_kernel 30 \
        > gpurun_out/${T}_tl16_timeline.txt 2>&1 ;;
    w2)
      # bench.py --gpus 2 started plainly: it launches its 2 ranks itself (VERDICT r05
      # item 1); both ranks on the one GPU over gloo (speed meaningless, n_gpus / dp2 checked)
      XA_BENCH_SHARED_DEVICE=1 run w2 400 python bench.py --gpus 2 --steps 10 --warmup 3 \
        --cpu-baseline-seconds 0
      XA_BENCH_SHARED_DEVICE=1 run w2c4 500 python bench.py --config c4 --gpus 2 --steps 2 \
        --warmup 1 --cpu-baseline-seconds 0 ;;
    c4dp) run_pytest c4dp 600 -s tests/test_gpu_dp.py -k cnn tests/test_gpu_configs.py::test_c4_ppo_cnn_128_env_shard ;;
    c5w2)
      # W = 2 rehearsal of the C5 data-parallel bench with both ranks on the one GPU (gloo;
      # the fused TD3 stages on 96 workgroups per rank so both ranks' launches are resident)
      XA_TD3_BLOCKS=96 XA_BENCH_SHARED_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0 run c5w2 300 \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29518 bench.py --config c5 --gpus 2 --steps 20 --warmup 3 \
        --cpu-baseline-seconds 0 ;;
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python bench.py --steps 20 --warmup 5 ;;
    ab)
      run ab_local 200 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0
      XA_PPO_LOCAL=0 run ab_spread 200 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0
      run ab_local2 200 python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0
      python tools/bench_brief.py gpurun_out/${T}_ab_*.out ;;
    prof)
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof \
        -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 5 \
        --cpu-baseline-seconds 0 > $R/gpurun_out/${T}_prof_bench.json 2>&1) || exit $? ;;
    pmc)
      TAG=${T} timeout -k 10 600 bash tools/gpurun_pmc_shapes.sh > gpurun_out/${T}_pmc.log 2>&1 || exit $?
      # the per-dispatch counter CSVs are too big to travel back: keep the per-launch summary
      cp profiles/traffic.json gpurun_out/${T}_traffic.json
      XA_TRAFFIC_OUT=gpurun_out/${T}_traffic.json python tools/pmc_traffic.py gpurun_out ${T}_n16 ${T}_n256 \
        > gpurun_out/${T}_traffic.log 2>&1
      find gpurun_out -name "*counter_collection.csv" -delete ;;
    variants)
      # A/B of the diagnostic variant libraries (tools/build_variant.py) against the product
      # build, interleaved: base, each variant, base again (bench lines without CPU baseline)
      B="python bench.py --steps 40 --warmup 5 --cpu-baseline-seconds 0 --no-secondary"
      run var_base1 200 $B
      for L in tools/diag_lib/libxa_*.so; do
        n=$(basename $L .so); n=${n#libxa_}
        [ "$n" = trace ] && continue
        run var_$n 200 $B --lib $L
      done
      run var_base2 200 $B
      python tools/bench_brief.py gpurun_out/${T}_var_*.out ;;
    profc3)
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_profc3 \
        -o run --output-format csv -- python $R/bench.py --config c3 --steps 30 --warmup 5 \
        --cpu-baseline-seconds 0 > $R/gpurun_out/${T}_profc3_bench.json 2>&1) || exit $?
      python tools/kernel_shapes.py gpurun_out/${T}_profc3/run_kernel_trace.csv 25 \
        > gpurun_out/${T}_profc3_shapes.txt 2>&1
      python tools/step_timeline.py gpurun_out/${T}_profc3/run_kernel_trace.csv conv_stack_bwd_reduce \
        > gpurun_out/${T}_profc3_timeline.txt 2>&1 ;;
    profc4)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_profc4 \
        -o run --output-format csv -- python $R/bench.py --config c4 --steps 2 --warmup 1 \
        --cpu-baseline-seconds 0 > $R/gpurun_out/${T}_profc4_bench.json 2>&1) || exit $?
      python tools/kernel_shapes.py gpurun_out/${T}_profc4/run_kernel_trace.csv 30 \
        > gpurun_out/${T}_profc4_shapes.txt 2>&1 ;;
    profc5)
      # C5 (TD3): the whole bench line, then one gradient step's launches on their own
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_profc5 \
        -o run --output-format csv -- python $R/bench.py --config c5 --steps 30 --warmup 5 \
        --cpu-baseline-seconds 0 > $R/gpurun_out/${T}_profc5_bench.json 2>&1) || exit $?
      (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_profc5g \
        -o run --output-format csv -- python $R/tools/td3_grad_steps.py 50 \
        > $R/gpurun_out/${T}_profc5g.log 2>&1) || exit $?
      python tools/kernel_shapes.py gpurun_out/${T}_profc5g/run_kernel_trace.csv 40 \
        > gpurun_out/${T}_profc5g_shapes.txt 2>&1
      python tools/step_timeline.py gpurun_out/${T}_profc5g/run_kernel_trace.csv td3_update 40 \
        > gpurun_out/${T}_profc5g_timeline.txt 2>&1
      python tools/step_timeline.py gpurun_out/${T}_profc5/run_kernel_trace.csv walker_step 30 \
        > gpurun_out/${T}_profc5_timeline.txt 2>&1 ;;
    td3gab)
      # fused TD3 gradient step: graph replay vs direct launch (XA_TD3_GRAPH), interleaved
      for r in 1 2; do
        run td3g_on$r 120 python tools/td3_grad_steps.py 100
        XA_TD3_GRAPH=0 run td3g_off$r 120 python tools/td3_grad_steps.py 100
        run c5g_on$r 300 python bench.py --config c5 --steps 30 --warmup 5 --cpu-baseline-seconds 0
        XA_TD3_GRAPH=0 run c5g_off$r 300 python bench.py --config c5 --steps 30 --warmup 5 --cpu-baseline-seconds 0
      done ;;
    stageab)
      # TD3 env-step rows in mapped host memory vs device rows + copies (XA_TD3_HOST_STAGE)
      for r in 1 2; do
        run c5s_on$r 300 python bench.py --config c5 --steps 30 --warmup 5 --cpu-baseline-seconds 0
        XA_TD3_HOST_STAGE=0 run c5s_off$r 300 python bench.py --config c5 --steps 30 --warmup 5 --cpu-baseline-seconds 0
      done ;;
    stepgab)
      # TD3 env step: hipGraph replay vs direct launches (XA_TD3_STEP_GRAPH), interleaved
      for r in 1 2 3; do
        run c5t_on$r 300 python bench.py --config c5 --steps 30 --warmup 5 --cpu-baseline-seconds 0
        XA_TD3_STEP_GRAPH=0 run c5t_off$r 300 python bench.py --config c5 --steps 30 --warmup 5 --cpu-baseline-seconds 0
      done ;;
    gs8ab)
      # PPO train steps per graph replay: XA_GRAPH_STEPS 8 (default) vs 4, interleaved
      B="python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --no-secondary"
      for r in 1 2 3; do
        run gs8_$r 200 $B
        XA_GRAPH_STEPS=4 run gs4_$r 200 $B
      done
      python tools/bench_brief.py gpurun_out/${T}_gs8_*.out gpurun_out/${T}_gs4_*.out ;;
    lgab)
      # DQN learner phase: hipGraph replay vs direct launches (XA_DQN_LEARN_GRAPH), C3 lines
      B="python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0"
      for r in 1 2; do
        run lg_on$r 300 $B
        XA_DQN_LEARN_GRAPH=0 run lg_off$r 300 $B
      done ;;
    xmapab)
      # fused dense dW + Adam: XCD-aware 1-D tile order vs the 2-D grid (XA_GEMM_ADAM_XMAP), C3
      B="python bench.py --config c3 --steps 30 --warmup 5 --cpu-baseline-seconds 0"
      for r in 1 2; do
        run xm_on$r 300 $B
        XA_GEMM_ADAM_XMAP=0 run xm_off$r 300 $B
      done ;;
    c2gs)
      # C2 train steps per graph replay: 8 (forced) vs the default (4 above 4096 env-steps)
      B="python bench.py --n-envs 256 --no-c2 --steps 24 --warmup 5 --cpu-baseline-seconds 0 --no-secondary --no-dynamics"
      for r in 1 2; do
        XA_GRAPH_STEPS=8 run c2gs8_$r 200 $B
        run c2gs4_$r 200 $B
      done
      python tools/bench_brief.py gpurun_out/${T}_c2gs*.out ;;
    c2g)
      # C2 update grid A/B: fewer workgroups with more tiles each (XA_PPO_MAX_BLOCKS)
      for G in ${C2_GS:-256 128}; do
        XA_PPO_MAX_BLOCKS=$G run c2g_$G 200 python bench.py --steps 30 --warmup 5 \
          --cpu-baseline-seconds 0 --no-secondary
      done
      python tools/bench_brief.py gpurun_out/${T}_c2g_*.out ;;
    td3pmc)
      # instruction-fetch and wait counters of the fused TD3 launch (one pass each)
      (cd /tmp && rocprofv3 -L > $R/gpurun_out/${T}_counters.txt 2>&1) || true
      (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
        SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM -d $R/gpurun_out/${T}_td3pmc1 \
        -o run --output-format csv -- python $R/tools/td3_grad_steps.py 10 \
        > $R/gpurun_out/${T}_td3pmc1.log 2>&1) || exit 3
      python tools/pmc_summary.py td3_update $(find gpurun_out/${T}_td3pmc1 -name "*counter_collection.csv") \
        > gpurun_out/${T}_td3pmc.txt
      (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS \
        -d $R/gpurun_out/${T}_td3pmc2 -o run --output-format csv -- python $R/tools/td3_grad_steps.py 10 \
        > $R/gpurun_out/${T}_td3pmc2.log 2>&1) || exit 4
      python tools/pmc_summary.py td3_update $(find gpurun_out/${T}_td3pmc2 -name "*counter_collection.csv") \
        >> gpurun_out/${T}_td3pmc.txt ;;
    smallm)
      run_pytest smallmtest 300 tests/test_gpu_layers.py -k "small_m or dense_input or layer_executor"
      run smallm 120 python tools/bench_smallm.py 16 64 128 336 ;;
    dprel) run dprel 700 bash tools/cnn_dp_rel.sh ;;
    sweep) run sweep 400 python tools/gemm_split_sweep.py 32 64 128 ;;
    c3host) run c3host 300 python tools/c3_host_profile.py ;;
    pollab)
      # poll-round sleep of the persistent update (XA_POLL_SLEEP variants,
      # tools/diag_lib/libxa_poll*.so) vs the product: bench lines (16-env + C2) and the
      # C2 update's FETCH_SIZE per launch
      B="python bench.py --steps 30 --warmup 5 --cpu-baseline-seconds 0 --no-secondary"
      run poll_base 200 $B
      for L in tools/diag_lib/libxa_poll*.so; do
        n=$(basename $L .so); n=${n#libxa_}
        run poll_$n 200 $B --lib $L
      done
      python tools/bench_brief.py gpurun_out/${T}_poll_*.out
      for L in product tools/diag_lib/libxa_poll*.so; do
        n=$(basename $L .so); n=${n#libxa_}
        LIBARG=""; [ "$L" != product ] && LIBARG="--lib $R/$L"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/${T}_pollpmc_$n \
          -o run --output-format csv -- python $R/bench.py --n-envs 256 --no-c2 --steps 2 --warmup 1 \
          --cpu-baseline-seconds 0 --no-graph --no-secondary $LIBARG \
          > $R/gpurun_out/${T}_pollpmc_$n.log 2>&1) || exit 7
        echo "== $n" >> gpurun_out/${T}_pollpmc.txt
        python tools/pmc_summary.py ppo_update $(find gpurun_out/${T}_pollpmc_$n -name "*counter_collection.csv") \
          >> gpurun_out/${T}_pollpmc.txt
        find gpurun_out/${T}_pollpmc_$n -name "*counter_collection.csv" -delete
      done ;;
    c3) run c3 300 python bench.py --config c3 --steps 30 --warmup 5 ;;
    c4) run c4 400 python bench.py --config c4 --steps 4 --warmup 1 ;;
    c5) run c5 300 python bench.py --config c5 --steps 30 --warmup 5 ;;
    acer) run acer 300 python bench.py --config acer --steps 10 --warmup 2 ;;
    trpo) run trpo 300 python bench.py --config trpo --steps 10 --warmup 2 ;;
    stamps) run stamps 200 python tools/diag_ppo_update.py --no-build ;;
    trace)
      run trace 200 python tools/trace_ppo_update.py --no-build 16 256
      run trace_spread 200 python tools/trace_ppo_update.py --no-build --spread 16 ;;
    icache)
      # instruction-cache counters of the 16-env update (one counter per pass)
      (cd /tmp && rocprofv3 -L > $R/gpurun_out/${T}_counters.txt 2>&1) || true
      for c in $(grep -oE '\bSQC?_(ICACHE|IFETCH|INST_CACHE)[A-Z_]*' gpurun_out/${T}_counters.txt | sort -u | head -4); do
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $c -d $R/gpurun_out/${T}_pmc_$c -o run \
          --output-format csv -- python $R/bench.py --n-envs 16 --no-c2 --steps 2 --warmup 1 \
          --cpu-baseline-seconds 0 --no-graph > $R/gpurun_out/${T}_pmc_$c.log 2>&1) || exit $?
      done ;;
    probe) run probe 120 ./tools/probe/tile_probe 200 ;;
    gemm)
      # the GEMM tests, small-M timings, and PMC passes on the M = 64 / 336 dense dX
      run_pytest gemm 300 tests/test_gpu_layers.py
      run smallm 120 python tools/bench_smallm.py 4 16 64 128 336
      for B in 64 336; do
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
          SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/${T}_gpmc/p1_$B -o run --output-format csv \
          -- python $R/tools/gemm_one.py 'dense dX' 10 $B > $R/gpurun_out/${T}_gpmc_p1_$B.log 2>&1) || exit 3
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM \
          SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAVES \
          -d $R/gpurun_out/${T}_gpmc/p2_$B -o run --output-format csv \
          -- python $R/tools/gemm_one.py 'dense dX' 10 $B > $R/gpurun_out/${T}_gpmc_p2_$B.log 2>&1) || exit 4
        python tools/pmc_summary.py 'gemm_' $(find gpurun_out/${T}_gpmc/p1_$B gpurun_out/${T}_gpmc/p2_$B \
          -name "*counter_collection.csv") > gpurun_out/${T}_gemm_pmc_M$B.txt
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
