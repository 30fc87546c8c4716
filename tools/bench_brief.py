"""One line per bench JSON file: value, ms per step, update / rollout launch times (16 envs
and C2), the dominant kernel's roofline fraction and traffic."""
import json
import sys

for path in sys.argv[1:]:
    try:
        r = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as exc:  # noqa: BLE001
        print(f'{path}: unreadable ({exc})')
        continue
    c2 = r.get('c2') or {}
    rl, c2rl = r.get('roofline') or {}, c2.get('roofline') or {}
    print(f'{path}: {r["value"] / 1e6:.3f} M/s {r["ms_per_step"]:.4f} ms '
          f'(update {rl.get("launch_ms")} rollout {(r.get("rollout_roofline") or {}).get("launch_ms")}) | '
          f'C2 {c2.get("value", 0) / 1e6:.2f} M/s {c2.get("ms_per_step")} ms '
          f'(update {c2rl.get("launch_ms")})')
