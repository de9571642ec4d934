#!/usr/bin/env python3
"""Per-step device time of a one-process kernel trace with the streams' overlap: the union of the kernels' [start, end)
intervals in each step (steps split at each launch of a marker kernel), beside the plain sum of their durations.
    python3 profiles/busy_union.py TRACE_DIR [--marker k_raw_count] [--skip 1]"""
import argparse
import collections
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--marker', default='k_raw_count')
    ap.add_argument('--skip', type=int, default=1, help='leading steps dropped (setup, first launch)')
    ap.add_argument('--exclude', default='', help='regex of kernels left out (e.g. rccl: world-1 self copies)')
    ap.add_argument('--top', type=int, default=0, help='per-kernel sums of the last step, largest first')
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, '**', '*kernel_trace.csv'), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sb::', '')
        if a.exclude and re.search(a.exclude, n):
            continue
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), n))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].startswith(a.marker)]
    out = []
    for s0, s1 in zip(starts, starts[1:]):
        seg = rows[s0:s1]
        tot = sum(e - b for b, e, _ in seg)
        busy, cur_b, cur_e = 0, None, None
        for b, e, _ in seg:
            if cur_e is None or b > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_b
                cur_b, cur_e = b, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_b
        out.append((tot / 1e6, busy / 1e6, (seg[-1][1] - seg[0][0]) / 1e6))
    for i, (t, b, sp) in enumerate(out):
        print(f'step {i}: kernels summed {t:.3f} ms, busy (union) {b:.3f} ms, span {sp:.3f} ms' +
              ('  (skipped)' if i < a.skip else ''))
    if a.top and len(starts) > 1:
        agg = collections.Counter()
        for b, e, n in rows[starts[-2]:starts[-1]]:
            agg[n] += (e - b) / 1e6
        print('last step:', {k: round(v, 3) for k, v in agg.most_common(a.top)})
    keep = out[a.skip:]
    if keep:
        print(f'mean over {len(keep)} steps: summed {sum(x[0] for x in keep) / len(keep):.3f} ms, '
              f'busy {sum(x[1] for x in keep) / len(keep):.3f} ms, span {sum(x[2] for x in keep) / len(keep):.3f} ms')


if __name__ == '__main__':
    main()
