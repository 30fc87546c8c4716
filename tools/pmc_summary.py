"""Per-dispatch averages of rocprofv3 --pmc counters for the kernels whose name contains a
pattern. usage: python tools/pmc_summary.py <pattern> <run_counter_collection.csv>..."""
import csv
import sys
from collections import defaultdict


def main(pattern, *files):
    tot = defaultdict(float)
    disp = defaultdict(set)
    name = None
    for f in files:
        for row in csv.DictReader(open(f)):
            if pattern not in row['Kernel_Name']:
                continue
            name = row['Kernel_Name']
            tot[row['Counter_Name']] += float(row['Counter_Value'])
            disp[row['Counter_Name']].add((f, row['Dispatch_Id']))
    print(f'# {name}')
    for k in sorted(tot):
        print(f'{k:28s} {tot[k] / max(len(disp[k]), 1):16.0f}  (per dispatch, {len(disp[k])} dispatches)')


if __name__ == '__main__':
    main(*sys.argv[1:])
