"""CPU tests of bench.py's multi-rank plumbing: `bench.py --gpus N`
started as a plain process launches N ranks itself (torch.distributed.run, 127.0.0.1), and a
rank whose WORLD_SIZE differs from --gpus refuses to report. XA_BENCH_LAUNCH_CHECK=1 makes
every rank stop after the process-group setup (gloo, no device) and rank 0 print the line's
n_gpus / parallelism fields."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, extra_env=None):
    env = dict(os.environ, XA_BENCH_LAUNCH_CHECK='1', MASTER_ADDR='127.0.0.1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, str(ROOT / 'bench.py'), *args], env=env,
                          capture_output=True, text=True, timeout=240)


def _json_lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith('{')]


@pytest.mark.parametrize('config', ['c2', 'c4', 'c5'])
def test_gpus_2_launches_two_ranks(config):
    r = _run(['--gpus', '2', '--config', config])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line['n_gpus'] == 2 and line['parallelism'] == 'dp2'
    assert line['rank_sum'] == 1 and line['config'] == config
    assert 'launching 2 ranks' in r.stderr


def test_gpus_1_runs_in_process():
    r = _run(['--gpus', '1'])
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line['n_gpus'] == 1 and line['parallelism'] == 'dp1'
    assert 'launching' not in r.stderr


def test_world_size_mismatch_refuses():
    r = _run(['--gpus', '4'], {'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert r.returncode != 0
    assert 'WORLD_SIZE 1' in r.stderr
    assert not _json_lines(r.stdout)
