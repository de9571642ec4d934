#!/usr/bin/env python3
"""Per-step HBM traffic of a world > 1 kernel from profiles/collect_r4_mig_pmc.sh (rank 0 and rank 1).

The timed steps are the last --steps of the bench run; a step's key pass is P launches of the kernel (its
exchange parts), so the per-step figures sum P consecutive dispatches: P = dispatches per step found from the
trace (dispatches of the kernel between consecutive k_mig_digit / k_raw_count launches).  Traffic per the
guide (MI355X_MICROARCH.md HBM section): hbm = (2 * FETCH_SIZE + WRITE_SIZE) KiB — the doubling calibrated for
random 16-B loads too by profiles/micro/fetchcal.hip (profiles/micro/r4_fetchcal.txt).
"""
import argparse
import csv
import glob
import json
import os
import re


def short(name):
    m = re.match(r'(?:void )?(?:sb::)?([A-Za-z_0-9]+(?:<[^>]*>)?)', name)
    return m.group(1) if m else name[:40]


def rows(d, counter=None):
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv' if counter else '*kernel_trace.csv'), recursive=True)
    out = []
    for r in csv.DictReader(open(f[0])):
        if counter and r['Counter_Name'] != counter:
            continue
        out.append((short(r['Kernel_Name']), int(r['Start_Timestamp']), int(r['End_Timestamp']),
                    float(r['Counter_Value']) if counter else None))
    out.sort(key=lambda x: x[1])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--kernel', default='k_mkeys_a')
    ap.add_argument('--steps', type=int, default=4)
    ap.add_argument('--out')
    a = ap.parse_args()
    res = {'kernel': a.kernel, 'steps': a.steps, 'ranks': {}}
    for r in (0, 1):
        tr = rows(os.path.join(a.dir, 'trace', f'r{r}'))
        cut = 'k_mig_digit' if any(x[0] == 'k_mig_digit' for x in tr) else 'k_raw_count'
        idx = [i for i, x in enumerate(tr) if x[0] == cut]
        last = tr[idx[-a.steps]:]
        k = [x for x in last if x[0] == a.kernel]
        P = max(1, round(len(k) / a.steps))
        ns = sum(x[2] - x[1] for x in k) / a.steps
        out = {'launches_per_step': P, 'device_ms_per_step': ns / 1e6}
        for name, ctr in (('fetch', 'FETCH_SIZE'), ('write', 'WRITE_SIZE'), ('tcc', 'TCC_HIT_sum'), ('tcc', 'TCC_MISS_sum')):
            v = [x[3] for x in rows(os.path.join(a.dir, name, f'r{r}'), ctr) if x[0] == a.kernel]
            out[ctr] = sum(v[-P * a.steps:]) / a.steps
        out['hbm_bytes_per_step'] = (2 * out['FETCH_SIZE'] + out['WRITE_SIZE']) * 1024
        out['tcc_hit_rate'] = out['TCC_HIT_sum'] / max(1.0, out['TCC_HIT_sum'] + out['TCC_MISS_sum'])
        out['traffic_GBps'] = out['hbm_bytes_per_step'] / (ns * 1e-9) / 1e9 if ns else None
        res['ranks'][r] = out
        print(f'rank {r}: {a.kernel} x{P}/step {ns / 1e6:.3f} ms/step, HBM {out["hbm_bytes_per_step"] / 1e9:.3f} GB/step '
              f'({out["traffic_GBps"]:.0f} GB/s), L2 hit {out["tcc_hit_rate"]:.3f}')
    m = {k: (res['ranks'][0][k] + res['ranks'][1][k]) / 2 for k in ('device_ms_per_step', 'hbm_bytes_per_step', 'tcc_hit_rate')}
    res['mean'] = m
    res['pmc'] = {a.kernel: {'hbm_bytes_per_step': m['hbm_bytes_per_step'], 'device_ms_per_step': m['device_ms_per_step'],
                             'tcc_hit_rate': m['tcc_hit_rate'], 'world': 2}}
    if a.out:
        json.dump(res, open(a.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
