"""Turn the rocprofv3 PMC passes (tools/gpurun_pmc_shapes.sh, run by `tools/gpu_steps.sh pmc`) into
profiles/traffic.json: HBM bytes per launch of the hot kernels, keyed per workload shape
(`<kernel>_<tag>`, e.g. ppo_update_n16) when the passes ran per shape. FETCH_SIZE / WRITE_SIZE are in KB; on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM), so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores."""
import csv
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
KERNELS = {'ac_grad': 'ac_grad_kernel<4, 2>', 'rollout': 'replay_rollout_kernel<4, 2>',
           'grad_reduce': 'grad_reduce_kernel', 'minibatch': 'minibatch_kernel',
           'ppo_update': 'ppo_update_kernel<4, 2,'}


def per_kernel(counter, src):
    files = sorted(Path(src).rglob('*counter_collection.csv'))
    if not files:
        raise SystemExit(f'no counter_collection.csv under {src}')
    vals = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get('Counter_Name') != counter:
                continue
            name = row.get('Kernel_Name', '')
            for key, pat in KERNELS.items():
                if pat in name:
                    vals[key].append(float(row['Counter_Value']))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def entries(fetch_dir, write_dir, suffix=''):
    fetch = per_kernel('FETCH_SIZE', fetch_dir)
    write = per_kernel('WRITE_SIZE', write_dir)
    res = {}
    for k in KERNELS:
        if k in fetch and k in write:
            f_kb, n = fetch[k]
            w_kb, _ = write[k]
            res[k + suffix] = {'bytes_per_launch': round((2 * f_kb + w_kb) * 1024),
                               'fetch_size_kb_raw': round(f_kb, 1), 'write_size_kb': round(w_kb, 1),
                               'dispatches': n,
                               'correction': 'FETCH_SIZE x 2 (gfx950 wide-read tally), KB = 1024 B'}
    return res, fetch


def main(out_dir='gpurun_out', *tags):
    """No tags: gpurun_out/pmc_{FETCH_SIZE,WRITE_SIZE} -> unsuffixed keys (round 1 layout).
    Tags (e.g. r02n_n16): gpurun_out/pmc_<tag>_{FETCH_SIZE,WRITE_SIZE} -> keys suffixed
    with the tag's last '_' field (ppo_update_n16). Merges into the existing file."""
    f_out = Path(os.environ.get('XA_TRAFFIC_OUT', ROOT / 'profiles' / 'traffic.json'))
    res = json.loads(f_out.read_text()) if f_out.exists() else {}
    if not tags:
        new, fetch = entries(Path(out_dir) / 'pmc_FETCH_SIZE', Path(out_dir) / 'pmc_WRITE_SIZE')
        res.update(new)
        if 'grad_reduce' in new:
            # calibration on a known byte count (MI355X_MICROARCH.md: other access widths
            # are uncalibrated): xa_grad_reduce reads exactly 256 rows x 4675 f32 with 4-B lanes
            known = 256 * 4675 * 4
            res['calibration'] = {'kernel': 'grad_reduce', 'known_read_bytes': known,
                                  'fetch_raw_bytes': round(fetch['grad_reduce'][0] * 1024),
                                  'factor': round(known / (fetch['grad_reduce'][0] * 1024), 3)}
    for tag in tags:
        suffix = '_' + tag.split('_')[-1]
        new, _ = entries(Path(out_dir) / f'pmc_{tag}_FETCH_SIZE',
                         Path(out_dir) / f'pmc_{tag}_WRITE_SIZE', suffix)
        for v in new.values():
            v['source'] = f'rocprofv3 --pmc passes {tag} (tools/gpurun_pmc_shapes.sh)'
        res.update(new)
    f_out.parent.mkdir(exist_ok=True)
    f_out.write_text(json.dumps(res, indent=1) + '\n')
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:])
