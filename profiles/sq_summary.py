#!/usr/bin/env python3
"""Per-kernel SQ counter summary from rocprofv3 --pmc runs (profiles/r5_c4_sq.sh): for each kernel, the
dispatch-averaged counters over its largest (saturated) dispatches, and the derived shares that say what binds it:
VALU issue share per SIMD (ACTIVE_INST_VALU x waves per SIMD / WAVE_CYCLES), wave-cycle split into
active / issue-stalled / parked (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md
PMC notes), instructions per wave by kind, and mean resident waves (LEVEL_WAVES / BUSY_CYCLES when collected).
    python3 profiles/sq_summary.py OUT_DIR [--kernel REGEX] [--min-grid N]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--kernel', default='.')
    ap.add_argument('--top', type=int, default=6, help='dispatches (largest grids) averaged per kernel')
    a = ap.parse_args()
    rx = re.compile(a.kernel)
    data = defaultdict(lambda: defaultdict(dict))   # kernel -> dispatch -> counter -> value
    grid = {}
    for f in glob.glob(os.path.join(a.dir, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sb::', '')
            if not rx.search(k):
                continue
            d = (f, r['Dispatch_Id'])
            data[k][d][r['Counter_Name']] = data[k][d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
            grid[(k, d)] = int(r['Grid_Size'])
    out = {}
    for k, ds in data.items():
        # counters from different passes live in different dispatches: average each counter over the largest
        # dispatches that carry it
        cs = defaultdict(list)
        for d, vals in ds.items():
            for c, v in vals.items():
                cs[c].append((grid[(k, d)], v))
        avg = {}
        for c, v in cs.items():
            v.sort()
            top = [x[1] for x in v if x[0] == v[-1][0]][-a.top:]
            avg[c] = sum(top) / len(top)
        w = avg.get('SQ_WAVES', 0) or 1
        row = {c: round(v, 1) for c, v in sorted(avg.items())}
        wc = avg.get('SQ_WAVE_CYCLES')
        if wc:
            for c in ('SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_ANY', 'SQ_WAIT_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS',
                      'SQ_ACTIVE_INST_SCA', 'SQ_ACTIVE_INST_VMEM', 'SQ_WAIT_INST_LDS'):
                if c in avg:
                    row['share_' + c[3:].lower()] = round(avg[c] / wc, 4)
        for c in ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR', 'SQ_INSTS_SMEM',
                  'SQ_INSTS_FLAT'):
            if c in avg:
                row['per_wave_' + c[9:].lower()] = round(avg[c] / w, 1)
        if 'SQ_LEVEL_WAVES' in avg and 'SQ_BUSY_CYCLES' in avg and avg['SQ_BUSY_CYCLES']:
            row['mean_resident_waves_per_SE_counter'] = round(avg['SQ_LEVEL_WAVES'] / avg['SQ_BUSY_CYCLES'], 2)
        out[k] = row
        print(f'== {k}')
        for c, v in row.items():
            print(f'   {c:40s} {v}')
    print(json.dumps(out))


if __name__ == '__main__':
    main()
