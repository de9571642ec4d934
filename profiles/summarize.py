#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run: per-kernel device time of the timed steps (kernel trace) and
HBM traffic per launch from the PMC passes.

Timed steps = the last `--steps` dispatches of each per-step kernel (bench.py runs setup turns,
warmup, then the timed steps).  Traffic per the guide (MI355X_MICROARCH.md §HBM; cdna_hip_programming
§7): FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced stream, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (the x2 is calibrated for
16 B/lane streams; other widths uncalibrated — stated beside the number).
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict

# kernels launched once per step on the saturated path (k_expand: the last launches include the
# pipelined expansion of the turn after the last timed one — one per step either way)
PER_STEP = ['k_expand<false>', 'k_expand<true>', 'k_count_lm', 'k_count_lm_tiles', 'k_tk_stage', 'k_tk_unstage', 'k_scan_apply', 'k_emit_w<1, false>', 'k_tk_count', 'k_tk_write', 'k_os_hist', 'k_os_pass',
            'k_gather_d', 'k_copy_idx', 'k_rexpand<1>', 'k_rexpand2<1>', 'k_remit<1>', 'k_rgather']


def short(name):
    m = re.match(r'(?:void )?(?:sb::)?([A-Za-z_0-9]+(?:<[^>]*>)?)', name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--out', required=True)
    ap.add_argument('--expand', default='k_expand',
                    help='name prefix of the per-step expansion kernel that delimits the timed turns '
                         '(k_rexpand for bench.py --realistic)')
    ap.add_argument('--edges', action='store_true',
                    help='the run used bench.py --lookahead-edges (round-2 accounting before session 4)')
    a = ap.parse_args()
    def load(path, counter=None):
        """[(name, start, end, value)] in dispatch order (value = counter value for PMC files)."""
        out = []
        for r in csv.DictReader(open(path)):
            if counter is not None and r['Counter_Name'] != counter:
                continue
            out.append((short(r['Kernel_Name']), int(r['Start_Timestamp']), int(r['End_Timestamp']),
                        float(r['Counter_Value']) if counter else None))
        out.sort(key=lambda x: x[1])
        return out

    def timed_window(recs):
        """Dispatches of the timed turns (one engine: bench.py --steps S --warmup 0).  Exact accounting
        (default): the last S expansions are the timed turns' own and everything from the first of them
        on is timed.  --edges: the first timed turn's expansion was launched inside the step before it
        and the last timed step launched the next one: the window lies between those two starts."""
        ex = [r for r in recs if r[0].startswith(a.expand)]
        if a.edges:
            t0, t1 = ex[-a.steps - 1][1], ex[-1][1]
        else:
            t0, t1 = ex[-a.steps][1], float('inf')
        return [r for r in recs if t0 <= r[1] < t1]

    rows = load(os.path.join(a.dir, 'trace', 'run_kernel_trace.csv'))
    by = defaultdict(list)
    for r in rows:
        by[r[0]].append(r[2] - r[1])
    kernels = {}
    for k, durs in by.items():
        kernels[k] = {'calls': len(durs), 'total_ns': sum(durs), 'avg_ns': sum(durs) / len(durs)}
    win = defaultdict(list)
    for r in timed_window(rows):
        win[r[0]].append(r[2] - r[1])
    timed = {}
    for k in PER_STEP:
        if k in win:
            d = win[k]
            timed[k] = {'launches': len(d), 'avg_ns': sum(d) / len(d), 'per_step_ns': sum(d) / a.steps}
    pmc = {}
    for kind, fn in (('FETCH_SIZE', 'pmc_fetch'), ('WRITE_SIZE', 'pmc_write'), ('TCC_HIT_sum', 'pmc_tcc'),
                     ('TCC_MISS_sum', 'pmc_tcc')):
        p = os.path.join(a.dir, fn, 'run_counter_collection.csv')
        if not os.path.exists(p):
            continue
        vals = defaultdict(list)
        for r in timed_window(load(p, kind)):
            vals[r[0]].append(r[3])
        for k, v in vals.items():
            unit = '_KiB_timed_avg' if kind.endswith('SIZE') else '_timed_avg'
            pmc.setdefault(k, {})[kind + unit] = sum(v) / len(v)
    for k, v in pmc.items():
        if 'FETCH_SIZE_KiB_timed_avg' in v and 'WRITE_SIZE_KiB_timed_avg' in v:
            v['hbm_bytes_per_launch'] = (2 * v['FETCH_SIZE_KiB_timed_avg'] + v['WRITE_SIZE_KiB_timed_avg']) * 1024
        if 'TCC_HIT_sum_timed_avg' in v and 'TCC_MISS_sum_timed_avg' in v:
            h, m = v['TCC_HIT_sum_timed_avg'], v['TCC_MISS_sum_timed_avg']
            v['tcc_hit_rate'] = h / (h + m) if h + m else None
    bench = None
    bp = os.path.join(a.dir, 'bench_trace.json')
    if os.path.exists(bp):
        try:
            bench = json.loads(open(bp).read().strip().splitlines()[-1])
        except Exception:
            bench = None
    out = {'source': a.dir, 'timed_steps': a.steps, 'timed': timed, 'pmc': pmc,
           'all_kernels': dict(sorted(kernels.items(), key=lambda kv: -kv[1]['total_ns'])), 'bench': bench}
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)
    for k, v in timed.items():
        t = pmc.get(k, {}).get('hbm_bytes_per_launch')
        print(f'{k:12s} avg {v["avg_ns"]/1e6:8.3f} ms   hbm/launch {t/1e9 if t else float("nan"):8.3f} GB')


if __name__ == '__main__':
    main()
