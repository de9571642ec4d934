#!/usr/bin/env python3
"""Per-kernel PMC table from profiles/counters.sh output: values of the largest (saturated) dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc'
data = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [(grid, value, dur_ns)]
for f in glob.glob(os.path.join(root, '*', 'run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sb::', '')
        data[k][r['Counter_Name']].append((int(r['Grid_Size']), float(r['Counter_Value']),
                                           int(r['End_Timestamp']) - int(r['Start_Timestamp']), r['Dispatch_Id']))
for k, cs in sorted(data.items()):
    print(f'== {k}')
    for c, v in sorted(cs.items()):
        v.sort(key=lambda x: (x[0], x[1]))
        big = [x for x in v if x[0] == v[-1][0]][-3:]   # largest grid: saturated launches
        vals = [x[1] for x in big]
        print(f'   {c:22s} {sum(vals) / len(vals):16.1f}   (n={len(v)}, grid={big[-1][0]}, dur_us={big[-1][2] / 1e3:.0f})')
