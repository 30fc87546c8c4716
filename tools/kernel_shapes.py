"""Per-(kernel, grid) time summary of a rocprofv3 kernel trace CSV.

usage: python tools/kernel_shapes.py gpurun_out/prof_c4/run_kernel_trace.csv [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
d = collections.defaultdict(list)
for r in rows:
    k = (r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:48],
         r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'], r['Workgroup_Size_X'])
    d[k].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = sum(sum(v) for v in d.values())
print(f'total {tot / 1e6:.1f} ms over {len(rows)} dispatches')
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f'{sum(v) / 1e6:8.1f} ms n={len(v):5d} avg={sum(v) / len(v) / 1e3:8.1f} us  {k}')
