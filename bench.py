"""Benchmark: PPO train steps on PPO CartPole-v1 (MLP[64,64], n_steps=128, synthetic
observation replay), one process per GPU.

    python bench.py --gpus N --steps K --warmup W
    (N>1 started plainly: bench.py starts the N ranks itself under torch.distributed.run,
    one process per GPU, before any GPU call; under an external
    `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...` it runs as
    one rank and checks WORLD_SIZE == N)

A step = one PPO train_step: fused rollout of n_envs x 128 steps (+GAE) and 4 epochs x 4
minibatches (shuffle, forward, clipped loss, backward, global-norm clip, Keras Adam; one
persistent launch on one GPU, all-reduce of the gradient when N>1).
`value` = the metric's 16-env workload (BASELINE metric "PPO 16-env"); the line's `c2`
object = BASELINE configs[1] (256 envs per GPU). Weak scaling: every rank owns its envs;
--global-envs N splits N envs over the ranks instead (strong scaling). At N = 1 the same
line also carries compact `c3` / `c4` / `c5` objects (BASELINE configs[2..4]: value, ms per
step, dominant-kernel roofline, a few-second CPU-port baseline); --config c3|c4|c5|trpo|acer
prints a full line for one of them. Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = 'env-steps/sec/GPU (PPO 16-env) + update ms; 1/2/4/8 MI355X'
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA dense peak (= vector peak)
# rollout kernel algorithmic bytes per env-step (replay env): reads obs 16 + state 16 +
# reward 4 + done 4; writes obs 16 + action/logp/value/entropy/reward/done/epret/return 32
ROLLOUT_BYTES_PER_ENV_STEP = 40 + 48
# CartPole-dynamics rollout: the env state lives in registers for the whole launch (read and
# written once per env); per env-step only the outputs: obs 16 + 32 as above
DYNAMICS_ROLLOUT_BYTES_PER_ENV_STEP = 48
# persistent update: the rollout buffers one epoch reads per sample (obs 16 B + action,
# old log-prob, old value, return 4 B each)
UPDATE_BYTES_PER_SAMPLE_EPOCH = 16 + 16


def mlp_fwd_flops(obs_dim=4, n_actions=2, hidden=64):
    """F = forward FLOPs per sample of the actor-critic MLP (9,088)."""
    return 2 * (obs_dim * hidden + hidden * hidden + hidden * (n_actions + 1))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--n-envs', type=int, default=16,
                   help='envs per GPU of the headline line (the metric is quoted on 16)')
    p.add_argument('--global-envs', type=int, default=0,
                   help='strong scaling: this many envs in all, split over the ranks (the '
                        'headline line then reports scaling "strong"; default: --n-envs per GPU)')
    p.add_argument('--no-secondary', dest='secondary', action='store_false',
                   help='skip the compact C3 / C4 / C5 objects of the default one-GPU line')
    p.add_argument('--no-c2', dest='c2', action='store_false',
                   help='skip the secondary BASELINE configs[1] (256 envs per GPU) measurement')
    p.add_argument('--no-dynamics', dest='dynamics', action='store_false',
                   help='skip the `dynamics` object (the headline workload on the CartPole-v1 '
                        'dynamics env: the step-loop rollout of an action-dependent env)')
    p.add_argument('--n-steps', type=int, default=128)
    p.add_argument('--t-rec', type=int, default=4096)
    p.add_argument('--seed', type=int, default=55)
    p.add_argument('--no-graph', action='store_true')
    p.add_argument('--cpu-baseline-seconds', type=float, default=15.0)
    p.add_argument('--cpu-threads', type=int, default=0)
    p.add_argument('--preprocess', action='store_true',
                   help='c3 / c4: AtariWrapper on device (xa_atari_step: frame skip 4, '
                        'gray + resize of synthetic raw 210x160 RGB frames) in every env step')
    p.add_argument('--lib', default=None,
                   help='diagnostic A/B only: load this variant library (tools/build_variant.py) '
                        'instead of xagents_amd/libxagents_hip.so')
    p.add_argument('--config', default='c2', choices=['c2', 'c3', 'c4', 'c5', 'trpo', 'acer'],
                   help='c2 (default, the BASELINE metric line); c3 DQN Pong-shaped, c4 PPO '
                        'CNN Breakout-shaped (global 1024 envs, strong scaling), c5 TD3')
    return p.parse_args()


def cpu_baseline(args, record, theta0):
    """The CPU port timed at 1 thread and at up to 16 threads (the box's share), the best of
    3 windows for each (other work on the shared host only ever slows a window down, so the
    best window is the stable estimate of the port's speed); the faster setting is the
    baseline, both are in `sample`."""
    sys.path.insert(0, str(ROOT / 'oracle'))
    import numpy as np
    import torch
    from cpu_ppo import time_cpu_baseline

    t_before = torch.get_num_threads()
    many = args.cpu_threads or min(16, os.cpu_count() or 1)
    window = max(args.cpu_baseline_seconds / 6.0, 1.0)
    res = {}
    for threads in sorted({1, many}):
        runs = [time_cpu_baseline(record, theta0, n_steps=args.n_steps, seconds=window,
                                  threads=threads) for _ in range(3)]
        vals = [v for v, _ in runs]
        res[threads] = (float(np.max(vals)), vals, runs[0][1])
    torch.set_num_threads(t_before)
    best = max(res, key=lambda t: res[t][0])
    value, _, info = res[best]
    per = '; '.join(f"{t} thread{'s' if t > 1 else ''}: best {res[t][0]:.0f} of "
                    f"[{', '.join(f'{v:.0f}' for v in res[t][1])}]" for t in sorted(res))
    return {
        'value': round(value, 1),
        'unit': 'env-steps/s',
        'cores': best,
        'kind': 'port',
        'sample': (f"PPO train steps of the same workload ({info['n_envs']} envs x "
                   f"{args.n_steps} steps, 4x4 minibatches) in 3 windows of {window:.1f} s per "
                   f"thread count ({per} env-steps/s; the faster is reported): per-env Python "
                   f"step_envs loop, torch-CPU f32 MLP + autograd, numpy GAE, Keras Adam "
                   f"(oracle/cpu_ppo.py)"),
    }


def load_traffic(key):
    """HBM bytes per launch from the committed PMC passes (profiles/traffic.json)."""
    f = ROOT / 'profiles' / 'traffic.json'
    if not f.exists():
        return None
    entry = json.loads(f.read_text()).get(key)
    return entry.get('bytes_per_launch') if entry else None


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started as a plain process: start N ranks under
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) as a CHILD process,
    before this process makes any GPU call (an exec after a GPU call is forbidden on this
    pool, and the ranks must own their devices), pass rank 0's one JSON line through and exit
    with the launcher's status. Under an external launcher (WORLD_SIZE set) nothing is
    spawned; `_dist_setup` then checks WORLD_SIZE == --gpus."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={args.gpus}', '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), str(ROOT / 'bench.py'), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')  # dmabuf IPC only on this driver
    print(f'bench: launching {args.gpus} ranks: {" ".join(cmd[1:])}', file=sys.stderr,
          flush=True)
    return subprocess.run(cmd, env=env, check=False).returncode


def _dist_setup(args=None):
    """One process per GPU over RCCL. Rehearsal knob for a one-GPU box only:
    XA_BENCH_SHARED_DEVICE=1 puts every rank on cuda:0 with a gloo group (RCCL refuses
    two ranks on one device); the peer all-reduce then runs between processes that
    share the GPU, so that run checks the N>1 code path, not its speed. The world must be
    the --gpus the line reports (SystemExit otherwise: a 1-GPU line from `--gpus 8` would be
    a wrong measurement, not a smaller one)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if args is not None and world != args.gpus:
        raise SystemExit(f'bench: --gpus {args.gpus} but the process group has WORLD_SIZE '
                         f'{world}')
    import torch
    import torch.distributed as dist
    if os.environ.get('XA_BENCH_LAUNCH_CHECK') == '1':
        # CPU check of the launcher path (tests/test_host.py): gloo, no device
        if world > 1:
            dist.init_process_group('gloo')
        return world, rank, torch.device('cpu')
    if os.environ.get('XA_BENCH_SHARED_DEVICE') == '1':
        local_rank = 0
        if world > 1:
            torch.cuda.set_device(0)
            dist.init_process_group('gloo')
    elif world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
    return world, rank, torch.device('cuda', local_rank)


def _max_over_ranks(x, device):
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if dist.get_backend() == 'gloo':
        t = t.cpu()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _timed(fn, steps, warmup, world):
    """W untimed + K timed calls bracketed by barrier + synchronize; max over ranks."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        el = _max_over_ranks(el, torch.device('cuda', torch.cuda.current_device()))
    return el


def secondary_cpu_baseline(args, kind, seconds=None, compact=False):
    """Bounded CPU sample of the C3 / C4 / C5 / TRPO / ACER workload (oracle/cpu_cnn.py,
    oracle/cpu_td3.py, oracle/cpu_trpo.py; kind "port"). compact: the few-second samples of
    the default line's c3 / c4 / c5 objects (C4: 16 steps per env instead of 128)."""
    seconds = args.cpu_baseline_seconds if seconds is None else seconds
    sys.path.insert(0, str(ROOT / 'oracle'))
    import numpy as np
    import torch
    import cpu_cnn
    from xagents_amd.envs import record_transitions
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    if kind == 'c4':
        n, T = 16, (16 if compact else 128)
        rec = record_transitions(n, 256, (84, 84, 1), np.uint8, seed=args.seed)
        value, info = cpu_cnn.time_cnn_ppo(rec, n_steps=T, seconds=seconds, threads=threads)
        sample = (f"{info['train_steps']} PPO-CNN train steps of {n} envs x {T} steps (4x4 "
                  f"minibatches of {n * T // 4}) in {info['seconds']:.1f} s: per-env Python step_envs "
                  f"loop, torch-CPU f32 Conv1D/dense + autograd, numpy GAE, Keras Adam "
                  f"(oracle/cpu_cnn.py); the GPU line runs 1024 envs")
    elif kind == 'c5':
        import cpu_td3
        n = 64
        rec = record_transitions(n, 4096, (24,), np.float32, seed=args.seed)
        np.random.seed(args.seed)
        value, info = cpu_td3.time_td3(rec, seconds=seconds, threads=threads)
        sample = (f"{info['train_steps']} TD3 train steps of {n} envs (gradient_steps 1 per "
                  f"finished episode, batch 64 from per-env ReplayBuffer2 rings) in "
                  f"{info['seconds']:.1f} s: per-env Python step_envs loop, torch-CPU f32 "
                  f"actor / twin critics + autograd, Keras Adam, Polyak (oracle/cpu_td3.py)")
    elif kind == 'trpo':
        import cpu_trpo
        n, T = 16, 512
        rec = record_transitions(n, 4096, (4,), np.float32, seed=args.seed)
        np.random.seed(args.seed)
        value, info = cpu_trpo.time_trpo(rec, seconds=seconds, threads=threads, n_steps=T)
        sample = (f"{info['train_steps']} TRPO train steps of {n} envs x {T} steps in "
                  f"{info['seconds']:.1f} s: per-env Python step_envs loop, numpy GAE, "
                  f"torch-CPU f32 actor / critic, autograd surrogate gradient, 10 CG "
                  f"iterations of double-backprop Fisher-vector products, line search, "
                  f"3 x 4 x 4 critic minibatches with Keras Adam (oracle/cpu_trpo.py); "
                  f"CartPole-shaped f32 transition replay")
    elif kind == 'acer':
        n, T = 16, 20
        rec = record_transitions(n, 256, (84, 84, 1), np.uint8, seed=args.seed)
        np.random.seed(args.seed)
        value, info = cpu_cnn.time_acer(rec, seconds=seconds, threads=threads, n_steps=T)
        sample = (f"{info['train_steps']} ACER train steps of {n} envs x {T} steps (fresh "
                  f"update + poisson(4) replays of random.sample'd trajectories) in "
                  f"{info['seconds']:.1f} s: per-env Python step_envs loop, torch-CPU f32 "
                  f"NatureCNN + autograd trust-region gradient, Python Retrace loop, Keras "
                  f"Adam, weight EMA (oracle/cpu_cnn.py)")
    else:
        n = 32
        rec = record_transitions(n, 256, (84, 84, 1), np.uint8, seed=args.seed)
        value, info = cpu_cnn.time_dqn(rec, seconds=seconds, threads=threads)
        sample = (f"{info['train_steps']} double-DQN train steps of {n} envs (batch 64 from "
                  f"per-env deques of 1000) in {info['seconds']:.1f} s: per-env Python "
                  f"step_envs loop, random.sample replay, torch-CPU f32 NatureCNN + autograd, "
                  f"Keras Adam (oracle/cpu_cnn.py)")
    torch.set_num_threads(threads)
    return {'value': round(value, 2), 'unit': 'env-steps/s', 'cores': info['threads'],
            'kind': 'port', 'sample': sample}


def _raw_kw(args, n):
    return {'t_raw_frames': 64 if n <= 64 else 16} if args.preprocess else {}


def _data_note(args, what):
    if args.preprocess:
        return ('synthetic: raw 210x160 RGB uint8 frames i.i.d. uniform (seed 55+rank) '
                'through AtariWrapper on device (frame skip 4, gray, resize 84x84)')
    return what


def dominant_kernel_roofline(executors, step):
    """Roofline of the CNN step's dominant launch: the recorded launch kind (dense dX, dense
    dW (+ Adam), the fused conv-stack forward / backward) with the largest total time in one
    more (eager) `step`, from HIP events recorded on the launch stream around each launch.
    HBM basis for launches that carry algorithmic bytes (the fused dense dW + Adam), MFMA f32
    otherwise (2 x MACs of the launch's GEMMs / convolutions)."""
    import torch
    timing = []
    for ex in executors:
        ex.timing = timing
    try:
        step()
        torch.cuda.synchronize()
    finally:
        for ex in executors:
            ex.timing = None
    tot = {}
    for name, e0, e1, fl, nb in timing:
        t = tot.setdefault(name, [0.0, 0, fl, nb])
        t[0] += e0.elapsed_time(e1)
        t[1] += 1
    if not tot:
        return None
    name, (ms_sum, cnt, fl, nb) = max(tot.items(), key=lambda kv: kv[1][0])
    ms = ms_sum / cnt
    share = ms_sum / sum(v[0] for v in tot.values())
    tf = fl / (ms * 1e-3) / 1e12
    mfma = {'achieved': round(tf, 3), 'peak': F32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(tf / F32_MFMA_PEAK_TFLOPS, 4)}
    note = (f'mean of {cnt} launches; {share:.0%} of the recorded launch time of the step '
            f'({", ".join(sorted(tot))})')
    if nb:
        gbs = nb / (ms * 1e-3) / 1e9
        return {'kernel': name, 'bound': 'hbm', 'achieved': round(gbs, 2),
                'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(gbs / HBM_PEAK_GBS, 4),
                'traffic': None, 'launch_ms': round(ms, 4), 'bytes_per_launch': int(nb),
                'mfma': mfma, 'note': 'algorithmic bytes (24 B per parameter: theta, m, v '
                'read and written; the layer input and output gradient read) / event time; '
                + note}
    return dict(kernel=name, bound='mfma', traffic=None, launch_ms=round(ms, 4),
                note='2 x MACs per launch / event time; ' + note, **mfma)


def dominant_gemm_roofline(executors, step):
    """Roofline of the GEMM launch shape with the largest total time in one more (eager)
    `step` (the layer executors' HIP event pairs on the launch stream)."""
    import torch
    timing = []
    for ex in executors:
        ex.timing = timing
    try:
        step()
        torch.cuda.synchronize()
    finally:
        for ex in executors:
            ex.timing = None
    tot = {}
    for name, e0, e1, fl, _ in timing:
        t = tot.setdefault((name, fl), [0.0, 0])
        t[0] += e0.elapsed_time(e1)
        t[1] += 1
    if not tot:
        return None
    (name, fl), (ms_sum, cnt) = max(tot.items(), key=lambda kv: kv[1][0])
    ms = ms_sum / cnt
    tf = fl / (ms * 1e-3) / 1e12
    share = ms_sum / sum(v[0] for v in tot.values())
    return {'kernel': f'xa_gemm {name} (MFMA f32)', 'bound': 'mfma', 'achieved': round(tf, 4),
            'peak': F32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(tf / F32_MFMA_PEAK_TFLOPS, 5), 'traffic': None,
            'launch_ms': round(ms, 5),
            'note': f'2 M N K FLOP per launch, mean of {cnt} launches; the largest total time '
                    f'of the GEMM shapes in a gradient step ({share:.0%} of the GEMM time; the '
                    f'step is launch-bound at batch 64)'}


def fused_td3_roofline(agent, launches=10):
    """Roofline of the fused TD3 gradient step (xa_td3_update, one persistent launch per
    gradient step): HIP event pairs on the launch stream around `launches` eager launches
    (gradient_steps 1: every step updates the actor)."""
    import numpy as np
    import torch
    agent.fused_timing = []
    try:
        for _ in range(launches):
            agent.update_weights(1)
        torch.cuda.synchronize()
        rows = list(agent.fused_timing)
    finally:
        agent.fused_timing = None
    # one gradient step's launch time: one launch, or the sum of its data-parallel stages
    # (the collectives between them excluded)
    ms = float(np.mean([sum(e0.elapsed_time(e1) for e0, e1 in evs) for _, evs in rows]))
    pol = sum(p for p, _ in rows) / len(rows)
    stages = len(rows[-1][1])
    flops = pol * agent.fused_step_flops(True) + (1 - pol) * agent.fused_step_flops(False)
    nbytes = pol * fused_td3_bytes(agent, True) + (1 - pol) * fused_td3_bytes(agent, False)
    tf = flops / (ms * 1e-3) / 1e12
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {'kernel': 'xa_td3_update (one persistent launch per gradient step: twin critics, '
                      'TD head, backward, Adam, actor update, Polyak)', 'bound': 'hbm',
            'achieved': round(gbs, 3), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 5), 'traffic': None,
            'launch_ms': round(ms, 5), 'bytes_per_launch': int(nbytes),
            'mfma': {'achieved': round(tf, 4), 'peak': F32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                     'frac': round(tf / F32_MFMA_PEAK_TFLOPS, 5),
                     'flops_per_launch': int(flops)},
            'note': f'HBM basis (SURVEY 8d C5): algorithmic bytes of one gradient step at batch '
                    f'{agent.batch_size} (theta / m / v / gradient of every trained network '
                    f'7 x 4 B x P, every target network read, + written on policy steps, the '
                    f'sampled batch gathered and written) / the mean of {len(rows)} '
                    f'event-timed launches; MFMA basis (2 M N K FLOP of every GEMM) under '
                    f'"mfma"; latency-bound (5 / 10 grid barriers between the 6 / 11 phases '
                    f'of a critic / policy step)' + (
                        f'; data parallel: the {stages} stage launches of a step summed, the '
                        f'gradient all-reduces between them excluded' if stages > 1 else '')}


def fused_td3_bytes(agent, policy=True):
    """Algorithmic HBM bytes of one DDPG / TD3 gradient step: the trained
    networks' theta, m, v read and written and their raw gradient written and read back
    (7 x 4 B per parameter: the critics every step, the actor on policy steps); the target
    networks read by the target forwards (target actor, target critics) and, on policy
    steps, written by the Polyak sync; the sampled batch (s, s', a, r, d) read from the rings
    and written for the caller."""
    nc = 2 if hasattr(agent, 'critic2') else 1
    pa, pc = agent.actor.n_params, agent.critic.n_params
    trained = nc * pc + (pa if policy else 0)
    targets = (pa + nc * pc) * (8 if policy else 4)
    batch = agent.batch_size * (2 * agent.S + agent.A + 2) * 4 * 2
    return 7 * 4 * trained + targets + batch


def launch_check(args):
    """XA_BENCH_LAUNCH_CHECK=1: the rank / world plumbing of an N-rank line without a GPU
    (every rank all-reduces its rank over gloo; rank 0 prints the line's n_gpus /
    parallelism fields)."""
    import torch
    import torch.distributed as dist
    world, rank, _ = _dist_setup(args)
    t = torch.tensor([float(rank)])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({'launch_check': True, 'n_gpus': world, 'parallelism': f'dp{world}',
                          'rank_sum': int(t.item()), 'config': args.config}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_offpolicy_and_cnn(args):
    """Secondary configs (TRPO, ACER); one JSON line each."""
    world, rank, device = _dist_setup(args)
    line = run_secondary(args, args.config, world, rank, device, args.steps, args.warmup,
                         args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def run_secondary(args, config, world, rank, device, steps, warmup, cpu_seconds, compact=False):
    """One secondary config's measurement (its JSON line as a dict)."""
    import numpy as np
    import torch
    from xagents_amd.envs import create_envs
    from xagents_amd.utils.common import create_buffers, create_model
    line = {'metric': METRIC, 'unit': 'env-steps/s', 'n_gpus': world, 'steps': steps,
            'warmup': warmup, 'higher_is_better': True, 'vs_baseline': None,
            'dtype': 'f32', 'cpu_baseline': None}
    if config == 'c3':
        from xagents_amd import DQN
        n = 32
        envs = create_envs('PongNoFrameskip-v4', n, args.preprocess, device=device,
                           seed=args.seed + rank, **_raw_kw(args, n))
        model = create_model(envs, 'dqn', 'model', seed=args.seed, device=device)
        bufs = create_buffers('dqn', 1_000_000, 64, n, initial_size=1_000_000)
        agent = DQN(envs, model, bufs, double=True, seed=args.seed, quiet=True,
                    epsilon_start=0.02, epsilon_end=0.02)
        t_fill = time.perf_counter()
        agent.fill_buffers()
        t_fill = time.perf_counter() - t_fill

        def step():
            agent.at_step_start()
            agent.train_step()
            agent.at_step_end()
        el = _timed(step, steps, warmup, world)
        env_steps = n * steps * world
        # one eager learner phase for the event pairs (the timed steps replay it as a graph)
        agent.use_graph = False
        rl = dominant_kernel_roofline([agent.ex_online], step)
        agent.use_graph = True
        if rl:
            line['roofline'] = rl
        line.update(scaling='weak', data=_data_note(
                        args, 'synthetic: Pong-shaped uint8 (84,84,1) frames i.i.d. uniform '
                        '(seed 55+rank), replay buffers pre-filled by device env steps'),
                    config={'workload': 'DQN/DDQN PongNoFrameskip-v4-shaped, 32 envs, NatureCNN '
                                        '(Conv1D cfg), ReplayBuffer1 1M total, buffer batch 64, '
                                        'double, epsilon 0.02 (BASELINE configs[2])',
                            'n_envs_per_gpu': n, 'batch': 64, 'replay_fill_s': round(t_fill, 2),
                            'parallelism': f'dp{world}'})
    elif config == 'c4':
        from xagents_amd import PPO
        n = 1024 // world
        envs = create_envs('BreakoutNoFrameskip-v4', n, args.preprocess, device=device,
                           seed=args.seed + rank, **_raw_kw(args, n))
        model = create_model(envs, 'ppo', 'model', seed=args.seed, device=device)
        agent = PPO(envs, model, n_steps=128, seed=args.seed, quiet=True)
        el = _timed(agent.fused_train_step, steps, warmup, world)
        env_steps = n * 128 * steps * world
        rl = dominant_kernel_roofline(agent.ex_chunks, agent.fused_train_step)
        if rl:
            line['roofline'] = rl
        line.update(scaling='strong', data=_data_note(
                        args, 'synthetic: Breakout-shaped uint8 (84,84,1) frames i.i.d. '
                        'uniform (seed 55+rank), random-init CNN'),
                    config={'workload': 'PPO BreakoutNoFrameskip-v4-shaped, 1024 envs global '
                                        'sharded over the GPUs, NatureCNN (Conv1D cfg), n_steps '
                                        '128, 4x4 minibatches (BASELINE configs[3])',
                            'n_envs_per_gpu': n, 'parallelism': f'dp{world}'})
    elif config == 'trpo':
        from xagents_amd import TRPO
        if world > 1:
            raise SystemExit('bench --config trpo runs on one GPU (TRPO is not data parallel)')
        n, T = 16, 512  # the reference's headline env count; trpo/cli.py n-steps default
        envs = create_envs('CartPole-v1', n, mode='transitions', device=device,
                           seed=args.seed, t_rec=4096)
        actor = create_model(envs, 'trpo', 'actor_model', seed=args.seed, device=device)
        critic = create_model(envs, 'trpo', 'critic_model', seed=args.seed + 1, device=device)
        agent = TRPO(envs, actor, critic, n_steps=T, seed=args.seed, quiet=True)
        el = _timed(agent.train_step, steps, warmup, world)
        env_steps = n * T * steps
        line.update(scaling='weak', data='synthetic: CartPole-v1 observation replay recorded '
                    'on the host (seed 55), random-init actor and critic', config={
                        'workload': 'TRPO CartPole-v1, 16 envs, n_steps 512, MLP actor / critic '
                                    '[64, 64] relu, CG 10 x FVP on every 5th state, line '
                                    'search, 3 x 4 x 4 critic minibatches (SURVEY 8f rank 2)',
                        'n_envs_per_gpu': n, 'parallelism': 'dp1'})
    elif config == 'acer':
        from xagents_amd import ACER
        n, T = 16, 20  # the headline env count; acer/cli.py n-steps default
        envs = create_envs('PongNoFrameskip-v4', n, args.preprocess, device=device,
                           seed=args.seed + rank, **_raw_kw(args, n))
        model = create_model(envs, 'acer', 'model', seed=args.seed, device=device)
        # 64 trajectories per env, replay from the first step (initial size 1 per env)
        bufs = create_buffers('acer', 64 * n, 1, n, initial_size=n)
        agent = ACER(envs, model, bufs, n_steps=T, seed=args.seed, quiet=True, grad_norm=10.0)
        np.random.seed(args.seed)
        el = _timed(agent.train_step, steps, warmup, world)
        env_steps = n * T * steps * world
        updates = int(agent.model.optimizer.iterations.item())
        rl = dominant_kernel_roofline(agent.ex_chunks, agent.train_step)
        if rl:
            line['roofline'] = rl
        line.update(scaling='weak', data=_data_note(
                        args, 'synthetic: Pong-shaped uint8 (84,84,1) frames i.i.d. uniform '
                        '(seed 55+rank), random-init CNN'),
                    config={'workload': 'ACER PongNoFrameskip-v4-shaped, 16 envs, n_steps 20, '
                                        'NatureCNN (Conv1D cfg, softmax actor + Q critic), '
                                        'trust region, replay ratio 4 (poisson), 64 '
                                        'trajectories per env (SURVEY 8f rank 2)',
                            'n_envs_per_gpu': n, 'parallelism': f'dp{world}',
                            'updates_per_step': round(updates / (steps + warmup), 2)})
    else:
        from xagents_amd import TD3
        n = max(64 // world, 1)
        envs = create_envs('BipedalWalker-v3', n, device=device, seed=args.seed + rank)
        kw = dict(seed=args.seed, device=device)
        actor = create_model(envs, 'td3', 'actor_model', **kw)
        critic = create_model(envs, 'td3', 'critic_model', **kw)
        bufs = create_buffers('td3', 1_000_000, 100, n, initial_size=n * 64)
        agent = TD3(envs, actor, critic, bufs, gradient_steps=1, seed=args.seed, quiet=True)
        agent.fill_buffers()
        # env steps with their done-triggered gradient steps, and one gradient step alone
        it0 = int(agent.critic.optimizer.iterations.item())
        el = _timed(agent.train_step, steps, warmup, world)
        grad_steps = int(agent.critic.optimizer.iterations.item()) - it0
        g_el = _timed(lambda: agent.update_weights(1), steps, warmup, world)
        env_steps = n * steps * world
        # one eager gradient step for the event pairs (the timed steps replay hipGraphs,
        # which carry no events)
        agent.use_graph = False
        if agent._fused_args() is not None:
            rl = fused_td3_roofline(agent)
        else:
            rl = dominant_gemm_roofline(
                [agent.ex_actor, agent.ex_target_actor, agent.ex_critic, agent.ex_critic2,
                 agent.ex_target_critic, agent.ex_target_critic2, agent.ex_critic_pi],
                lambda: agent.update_weights(1))
        agent.use_graph = True
        if rl:
            line['roofline'] = rl
        line.update(scaling='weak', data='synthetic: BipedalWalker-shaped f32 obs ~N(0,1) '
                    '(seed 55+rank)', config={
                        'workload': 'TD3 BipedalWalker-v3-shaped, 64 envs, ReplayBuffer2, '
                                    'per-buffer batch 1 (100 // 64), gradient_steps 1 '
                                    '(BASELINE configs[4])',
                        'n_envs_per_gpu': n, 'parallelism': f'dp{world}',
                        'gradient_step': (
                            'layer executor' if agent._fused_args() is None else
                            'xa_td3_update, one persistent launch' if world == 1 else
                            'xa_td3_update in 3 stages: critic gradients, all-reduce, critic '
                            'Adam + actor gradient, all-reduce, actor Adam'),
                        # the value depends on how often episodes end: every finished
                        # episode of the union triggers gradient_steps gradient steps
                        # (ddpg/agent.py:157-166)
                        'synthetic_episode_length': 'record dones ~ Bernoulli(1/200) per step '
                                                    '(Geometric, mean 200) + a forced terminal '
                                                    'at the record end (t_rec 256)',
                        'gradient_steps_per_env_step': round(
                            grad_steps / ((steps + warmup) * n * world), 5),
                        'gradient_steps_per_train_step': round(
                            grad_steps / (steps + warmup), 4)},
                    gradient_step_ms=round(g_el / steps * 1e3, 4))
    line['value'] = round(env_steps / el, 1)
    line['ms_per_step'] = round(el / steps * 1e3, 4)
    if rank == 0 and world == 1 and config in ('c3', 'c4', 'c5', 'trpo', 'acer') and \
            cpu_seconds > 0:
        line['cpu_baseline'] = secondary_cpu_baseline(args, config, cpu_seconds, compact)
    return line


# the default one-GPU line's compact secondary objects: (config, steps, warmup, CPU seconds)
SECONDARY = (('c3', 30, 5, 4.0), ('c4', 3, 1, 3.0), ('c5', 30, 5, 3.0))


def compact_secondaries(args, device):
    """C3 / C4 / C5 (BASELINE configs[2..4]) measured in the same run as the headline, each
    as a compact object: value, ms per step, the dominant kernel's roofline, a few-second
    CPU-port baseline. A failing config is reported as an error in its object."""
    import gc

    import torch
    out = {}
    for cfg, steps, warmup, cpu_s in SECONDARY:
        try:
            r = run_secondary(args, cfg, 1, 0, device, steps, warmup,
                              cpu_s if args.cpu_baseline_seconds > 0 else 0.0, compact=True)
            out[cfg] = {k: r[k] for k in ('value', 'unit', 'ms_per_step', 'scaling', 'steps',
                                          'warmup') if k in r}
            out[cfg]['workload'] = r['config']['workload']
            for k in ('synthetic_episode_length', 'gradient_steps_per_env_step',
                      'gradient_steps_per_train_step'):
                if k in r['config']:
                    out[cfg][k] = r['config'][k]
            out[cfg]['roofline'] = r.get('roofline')
            out[cfg]['cpu_baseline'] = r.get('cpu_baseline')
            if 'gradient_step_ms' in r:
                out[cfg]['gradient_step_ms'] = r['gradient_step_ms']
        except Exception as exc:  # noqa: BLE001 -- reported in the line, never hidden
            out[cfg] = {'error': f'{type(exc).__name__}: {exc}'}
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return out


def bench_ppo(args, world, rank, device, n_envs, env='replay'):
    """Time PPO train steps on n_envs CartPole envs per rank; returns the measurements and
    the per-kernel roofline of this workload. env 'replay': the synthetic observation replay
    of the metric (the record stream ignores the actions, so the rollout runs its T policy
    forwards as one batched launch, `replay_rollout_kernel`); 'dynamics': CartPole-v1
    dynamics on the device (`CartPoleVecEnv`, f64 as gym), whose next observation depends on
    the sampled action, so the rollout is the sequential step loop (`mlp_rollout_kernel`) --
    the rate a real device env gets."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from xagents_amd import PPO
    from xagents_amd.envs import CartPoleVecEnv, ReplayVecEnv, record_cartpole_replay
    from xagents_amd.utils.common import create_model

    if env == 'dynamics':
        record = None
        envs = CartPoleVecEnv(n_envs, seed=args.seed + rank, device=device)
    else:
        record = record_cartpole_replay(n_envs, args.t_rec, seed=args.seed + rank)
        envs = ReplayVecEnv('CartPole-v1', n_envs, device=device, record=record)
    model = create_model(envs, 'ppo', 'model', optimizer_kwargs=dict(learning_rate=7e-4),
                         seed=args.seed, device=device)
    theta0 = model.theta.cpu().numpy().copy()
    agent = PPO(envs, model, n_steps=args.n_steps, seed=args.seed, quiet=True,
                use_graph=not args.no_graph)
    if world > 1:
        dist.barrier()  # the data-parallel update's in-launch exchanges wait for every rank
    for _ in range(args.warmup):
        agent.train_step()
    transport = agent.check_peer_all_reduce()
    if transport == 'rccl' and world > 1:
        agent.train_step()  # re-capture on RCCL after a peer-path fallback
    for s in getattr(agent, '_graph_sizes', None) or [1]:
        agent.fused_train_steps(s)  # (each multi-step graph's first replay, untimed)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.fused_train_steps(args.steps)  # (groups of graph_steps() per graph replay)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the rollout / update split: the same K steps again with HIP events between the
    # phases, outside the timed region (an event record costs ~3 us of stream time)
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for k in range(args.steps):
        agent.fused_train_step(events[k])
    torch.cuda.synchronize()
    # per-kernel durations: HIP events on the launch stream around the rollout and the
    # update launches of 3 eagerly launched train steps right after the timed region
    ktimes = {}
    for _ in range(3):
        for k, v in agent.timed_train_step().items():
            ktimes.setdefault(k, []).extend(v)
    if world > 1:
        elapsed = _max_over_ranks(elapsed, device)
    agent._drain_episode_stats()
    T = args.n_steps
    B = n_envs * T
    mb = B // agent.mini_batches
    K = agent.ppo_epochs * agent.n_mb
    flops_sample = 3 * mlp_fwd_flops()  # forward + backward per sample
    out = {
        'n_envs': n_envs,
        'value': n_envs * T * args.steps * world / elapsed,
        'ms_per_step': elapsed / args.steps * 1e3,
        'rollout_ms': float(np.mean([e[0].elapsed_time(e[1]) for e in events])),
        'update_ms': float(np.mean([e[1].elapsed_time(e[2]) for e in events])),
        'transport': transport, 'graph': bool(agent.use_graph and agent._graph is not None),
        'graph_steps': getattr(agent, '_graph_S', 1) if agent._graph is not None else 0,
        'update_mode': agent.update_mode, 'record': record, 'theta0': theta0, 'agent': agent,
    }
    roll_ms = float(np.mean(ktimes['rollout']))
    if env == 'dynamics':
        per = DYNAMICS_ROLLOUT_BYTES_PER_ENV_STEP
        kname = 'xa_mlp_rollout (mlp_rollout_kernel<4,2>, CartPole-v1 dynamics step loop)'
        tkey = f'rollout_dyn_n{n_envs}'
        note = (f'latency-bound: one wave64 per env runs its {T} steps in order (policy '
                f'forward, categorical sample, f64 CartPole step: the next input depends on '
                f'the sampled action), heads / log-prob / entropy per 64-step chunk, fused '
                f'GAE; {per} algorithmic B/env-step x {B} env-steps per launch')
    else:
        per = ROLLOUT_BYTES_PER_ENV_STEP
        kname = 'xa_mlp_rollout (replay_rollout_kernel<4,2>)'
        tkey = f'rollout_n{n_envs}'
        note = (f'latency-bound: the replay records ignore the actions, so one 8-wave '
                f'workgroup per env runs its {T} policy forwards (+ the bootstrap row) as '
                f'independent 16-row MFMA tiles, then the step-order episode-return and '
                f'return chains; {per} algorithmic B/env-step x {B} env-steps per launch')
    roll_gbs = per * B / (roll_ms * 1e-3) / 1e9
    out['rollout_roofline'] = {
        'kernel': kname, 'bound': 'hbm',
        'achieved': round(roll_gbs, 3), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'frac': round(roll_gbs / HBM_PEAK_GBS, 6),
        'traffic': load_traffic(tkey), 'launch_ms': round(roll_ms, 5), 'note': note}
    if agent.update_mode == 'persistent':
        upd_ms = float(np.mean(ktimes['ppo_update']))
        flops = flops_sample * B * agent.ppo_epochs  # every sample once per epoch
        tf = flops / (upd_ms * 1e-3) / 1e12
        # SURVEY 8(d) HBM basis (north_star: "fraction of HBM roofline"): the rollout
        # buffers read once per epoch (obs 16 + action / log-prob / value / return 16 B per
        # sample) + the optimizer's 7 words per parameter per step (theta, m, v read and
        # written, the gradient read)
        P = agent.model.n_params
        alg_bytes = UPDATE_BYTES_PER_SAMPLE_EPOCH * B * agent.ppo_epochs + 7 * 4 * P * K
        gbs = alg_bytes / (upd_ms * 1e-3) / 1e9
        traffic = load_traffic(f'ppo_update_n{n_envs}')
        out['update_roofline'] = {
            'kernel': 'xa_ppo_update (ppo_update_kernel<4,2>, persistent)', 'bound': 'hbm',
            'achieved': round(gbs, 3), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 6), 'traffic': traffic,
            'algorithmic_bytes': alg_bytes,
            'traffic_ratio': round(traffic / alg_bytes, 3) if traffic else None,
            'launch_ms': round(upd_ms, 5),
            'mfma': {'achieved': round(tf, 3), 'peak': F32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                     'frac': round(tf / F32_MFMA_PEAK_TFLOPS, 5),
                     'flops': flops},
            'note': f'HBM basis: {UPDATE_BYTES_PER_SAMPLE_EPOCH} B/sample x {B} samples x '
                    f'{agent.ppo_epochs} epochs + 7 x 4 B x P = {P} x {K} optimizer steps; '
                    f'mfma: 3F = {flops_sample} FLOP/sample (fwd + bwd) per epoch; {K} '
                    f'optimizer steps of {mb} in ONE launch on {agent.update_blocks} '
                    f'workgroups; latency-bound (2 in-launch exchanges per optimizer step); '
                    f'launch_ms = HIP event pair on the launch stream around each launch of '
                    f'3 eager train steps; traffic = PMC FETCH_SIZE x 2 + WRITE_SIZE bytes per '
                    f'launch (profiles/traffic.json)'}
    else:
        grad_ms = float(np.mean(ktimes['ac_grad']))
        tf = flops_sample * mb / (grad_ms * 1e-3) / 1e12
        out['update_roofline'] = {
            'kernel': 'xa_ac_grad (ac_grad_kernel<4,2>, per-minibatch chain)', 'bound': 'mfma',
            'achieved': round(tf, 3), 'peak': F32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
            'frac': round(tf / F32_MFMA_PEAK_TFLOPS, 5),
            'traffic': load_traffic(f'ac_grad_n{n_envs}'), 'launch_ms': round(grad_ms, 5),
            'note': f'3F = {flops_sample} FLOP/sample x {mb} samples per launch, {K} launches '
                    f'per train step (data-parallel chain)'}
    return out


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit('--gpus must be >= 1')
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args))  # before anything touches the GPU
    if os.environ.get('XA_BENCH_LAUNCH_CHECK') == '1':
        return launch_check(args)
    if args.lib:
        from xagents_amd import _lib
        _lib._lib = _lib.load(args.lib)
    if args.config != 'c2':
        return bench_offpolicy_and_cnn(args)
    import torch.distributed as dist

    world, rank, device = _dist_setup(args)
    # headline: the metric's PPO CartPole-v1 16-env workload (BASELINE metric / configs[0]
    # shape) on the GPU; secondary: BASELINE configs[1] (256 envs per GPU); strong scaling
    # (--global-envs): the given env count split over the ranks
    if args.global_envs and args.global_envs % world:
        raise SystemExit(f'--global-envs {args.global_envs} is not divisible by {world} ranks')
    n_head = args.global_envs // world if args.global_envs else args.n_envs
    head = bench_ppo(args, world, rank, device, n_head)
    c2 = bench_ppo(args, world, rank, device, 256) if args.c2 and n_head != 256 else None
    # the same 16-env PPO on the CartPole-v1 dynamics env: the sequential step-loop rollout a
    # real (action-dependent) device env runs, beside the replay headline
    dyn = bench_ppo(args, world, rank, device, n_head, env='dynamics') if args.dynamics else None
    # BASELINE configs[2..4] as compact objects of the same one-GPU line
    sec = compact_secondaries(args, device) if world == 1 and args.secondary else {}

    if rank == 0:
        def dominant(r):
            # the kernel with the larger share of the step carries the line's roofline
            u, ro = r['update_roofline'], r['rollout_roofline']
            return dict(u) if u['launch_ms'] >= ro['launch_ms'] else dict(ro)

        line = {
            'metric': METRIC,
            'value': round(head['value'], 1),
            'unit': 'env-steps/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(head['ms_per_step'], 4),
            'higher_is_better': True,
            'scaling': 'strong' if args.global_envs else 'weak',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic: CartPole-v1 observation replay recorded on the host '
                    '(np.random.default_rng(55+rank)), random-init weights',
            'config': {
                'workload': (f'PPO CartPole-v1, {n_head} envs/GPU'
                             + (f' ({args.global_envs} in all)' if args.global_envs else '')
                             + f', MLP[64,64], n_steps={args.n_steps}, 4 epochs x 4 minibatches, '
                             f'synthetic obs replay' + (' (the metric\'s 16-env configuration)'
                                                        if n_head * world == 16 or
                                                        (n_head == 16 and not args.global_envs)
                                                        else '')
                             + '; the replay records ignore the actions, so the rollout runs '
                               'its policy forwards as one batched launch (the `dynamics` '
                               'object times the sequential step loop of an action-dependent '
                               'env)'),
                'n_envs_per_gpu': n_head,
                'n_steps': args.n_steps,
                'batch_per_gpu': n_head * args.n_steps,
                'minibatch_per_gpu': n_head * args.n_steps // 4,
                'ppo_epochs': 4,
                'parallelism': f'dp{world}',
                'graph': head['graph'],
                'train_steps_per_graph_replay': head['graph_steps'],
                'update': head['update_mode'],
                'allreduce': head['transport'],
            },
            'update_ms': round(head['update_ms'], 4),
            'rollout_ms': round(head['rollout_ms'], 4),
            'env_steps_per_sec_per_gpu': round(head['value'] / world, 1),
            'roofline': dominant(head),
            'update_roofline': head['update_roofline'],
            'rollout_roofline': head['rollout_roofline'],
        }
        if c2 is not None:
            line['c2'] = {
                'workload': 'PPO CartPole-v1, 256 envs/GPU, MLP[64,64], n_steps=128, 4x4 '
                            'minibatches of 8192, synthetic obs replay (BASELINE configs[1])',
                'value': round(c2['value'], 1), 'unit': 'env-steps/s',
                'ms_per_step': round(c2['ms_per_step'], 4),
                'update_ms': round(c2['update_ms'], 4), 'rollout_ms': round(c2['rollout_ms'], 4),
                'update': c2['update_mode'],
                'roofline': dominant(c2),
                'update_roofline': c2['update_roofline'],
                'rollout_roofline': c2['rollout_roofline'],
            }
        if dyn is not None:
            line['dynamics'] = {
                'workload': f'PPO CartPole-v1, {n_head} envs/GPU, MLP[64,64], n_steps='
                            f'{args.n_steps}, 4x4 minibatches, CartPole-v1 dynamics on the '
                            f'device (CartPoleVecEnv, f64 state as gym; the next observation '
                            f'depends on the sampled action, so the rollout is the sequential '
                            f'step loop)',
                'value': round(dyn['value'], 1), 'unit': 'env-steps/s',
                'ms_per_step': round(dyn['ms_per_step'], 4),
                'update_ms': round(dyn['update_ms'], 4),
                'rollout_ms': round(dyn['rollout_ms'], 4),
                'update': dyn['update_mode'],
                'roofline': dominant(dyn),
                'update_roofline': dyn['update_roofline'],
                'rollout_roofline': dyn['rollout_roofline'],
            }
        line.update(sec)
        if world == 1 and args.cpu_baseline_seconds > 0:
            line['cpu_baseline'] = cpu_baseline(args, head['record'], head['theta0'])
        else:
            line['cpu_baseline'] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        for r in (head, c2, dyn):
            if r is not None and r['agent'].peer is not None:
                r['agent'].peer.close()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
