"""Per-step timeline of a rocprofv3 kernel trace: steps are delimited by the launches of a
marker kernel (default clip_adam_kernel, the last launch of a DQN / CNN train step); prints the
median step span, kernel-busy time and launch count over the last N steps, then the last
step's launches (a step from the middle of the window) with the idle gap before each.
usage: python tools/step_timeline.py run_kernel_trace.csv [marker] [N]"""
import csv
import statistics
import sys


def main(path, marker='clip_adam_kernel', n=30):
    n = int(n)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    spans, busy, counts = [], [], []
    for a, b in zip(idx[-n - 1:-1], idx[-n:]):
        seg = rows[a + 1:b + 1]
        spans.append((int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3)
        # union of the launches' intervals (launches on two streams may overlap)
        t, u = int(rows[a]['End_Timestamp']), 0
        for r in seg:
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            if e > t:
                u += e - max(s, t)
                t = e
        busy.append(u / 1e3)
        counts.append(len(seg))
    print(f'{len(idx)} marker launches; last {len(spans)} steps: span {statistics.median(spans):.1f} us, '
          f'kernel busy {statistics.median(busy):.1f} us, {statistics.median(counts)} launches')
    k = len(idx) - 1 - len(spans) // 2  # a step from the middle of the window
    prev = int(rows[idx[k - 1]]['End_Timestamp'])
    for r in rows[idx[k - 1] + 1:idx[k] + 1]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        grid = r.get('Grid_Size_X') or r.get('Grid_Size') or ''
        print(f'  gap {(s - prev) / 1e3:6.1f}  dur {(e - s) / 1e3:7.1f}  {r["Kernel_Name"][:70]}  grid {grid}')
        prev = e


if __name__ == '__main__':
    main(*sys.argv[1:])
