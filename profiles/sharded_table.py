#!/usr/bin/env python3
"""Per-rank device time of the sharded step, by protocol phase, from profiles/collect_r3_sharded.sh traces.

Each rank's kernel trace (rocprofv3 --kernel-trace, one process per rank, SB_DIST_SERIALIZE=1 so every
kernel ran alone on the device) is cut into steps at its k_expand<true> launches (a step's expansion is
launched at the end of the previous step, its first kernel k_raw_count; the timed window is the last --steps).  Kernels are
assigned to phases by name, k_part_* by position (before the apply: the owner partition of the records;
after: the rebalance of the kept records).  Prints a table (ms per step, mean over the timed steps and
ranks, and the slowest rank) and writes it as JSON with --out.
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict

PHASES = [
    ('parent migration (card-set owners)', r'^k_mig_digit|^k_mig_unpack|^k_part_scatter<4>|^k_mig_place'),
    ('expand', r'^k_expand<true>|^k_keys_a|^k_mkeys_a|^k_ks_counts|^k_raw_count|^k_scan_(tiles|reduce|apply)$'),
    ('record pack', r'^k_keys_b|^k_mkeys_b'),
    ('owner partition', r'^k_part_|^k_chunk_counts'),
    ('owner claims', r'^k_own_|^k_mig_map|^k_mig_claim|^k_claim_goc'),
    ('answer bits', r'^k_(un)?pack_bits'),
    ('apply', r'^k_apply_w|^k_count_masks|^k_counts_i64|^k_total_i64'),
    ('noise (side stream)', r'^k_mt_'),
    ('emit', r'^k_emit_w|^k_oe_(rowcnt|groups|pack|fix)'),
    ('joint select', r'^k_ds_|^k_tk_|^k_oe_ties'),
    ('rebalance partition', r'^k_dest|^k_part_|^k_gkr_groups|^k_gkr_layout|^k_gkr_scatter|^k_chunk_counts'),
    ('receive sort + gather', r'^k_recv_|^k_iota|^k_os_|^k_fx_|^k_copy_idx|^k_oe_recv|^k_oe_compose|^k_oe_merge|'
                              r'^k_gkr_flags|^k_gkr_expand|^k_gkr_cnt'),
]


def short(name):
    m = re.match(r'(?:void )?(?:sb::)?([A-Za-z_0-9]+(?:<[^>]*>)?)', name)
    return m.group(1) if m else name[:40]


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((short(r['Kernel_Name']), int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    rows.sort(key=lambda x: x[1])
    return rows


def find_trace(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith('kernel_trace.csv'):
                return os.path.join(root, f)
    raise FileNotFoundError(d)


def overlap_flags(rows, others):
    """True for each kernel of `rows` that overlaps a kernel of another rank in time (the serialisation lock
    does not cover everything a process puts on the device), using the merged intervals of `others`."""
    iv = sorted((a, b) for _, a, b in others)
    merged = []
    for a, b in iv:
        if merged and a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    import bisect
    starts = [m[0] for m in merged]
    out = []
    for _, a, b in rows:
        i = bisect.bisect_right(starts, b) - 1
        out.append(i >= 0 and merged[i][1] > a)
    return out


def rank_table(rows, steps, ovl=None, cap=None):
    """ovl: per-row overlap flags; an overlapped kernel counts at the median of its clean instances.  cap: per
    kernel name, an upper bound on one instance's duration (the robust table: a launch that took longer than 1.5x
    the median of its instances over all ranks waited on another process's work on the shared GPU)."""
    clean = defaultdict(list)
    if ovl is not None:
        for (name, t0, t1), o in zip(rows, ovl):
            if not o:
                clean[name].append((t1 - t0) / 1e6)
    med = {k: sorted(v)[len(v) // 2] for k, v in clean.items()}
    # each step's expansion starts with k_raw_count; with card-set ownership its front (the parents' owner
    # digits, launched at the previous step's end) with k_mig_digit
    cut = 'k_mig_digit' if any(r[0] == 'k_mig_digit' for r in rows) else 'k_raw_count'
    ex = [i for i, r in enumerate(rows) if r[0] == cut]
    if len(ex) < steps:
        raise RuntimeError(f'only {len(ex)} expansions in the trace')
    starts = ex[-steps:] + [len(rows)]
    per = defaultdict(float)
    unknown = defaultdict(float)
    spans = []
    for s in range(steps):
        seg = rows[starts[s]:starts[s + 1]]
        segovl = ovl[starts[s]:starts[s + 1]] if ovl is not None else [False] * len(seg)
        applied = False
        for (name, t0, t1), o in zip(seg, segovl):
            dt = (t1 - t0) / 1e6
            if o and name in med:
                dt = med[name]
            if cap is not None and name in cap:
                dt = min(dt, cap[name])
            if name.startswith('k_apply_w'):
                applied = True
            ph = None
            for p, rx in PHASES:
                if re.search(rx, name):
                    if p == 'owner partition' and applied:
                        continue
                    if p == 'rebalance partition' and not applied:
                        continue
                    ph = p
                    break
            if ph is None:
                unknown[name] += dt
            else:
                per[ph] += dt
        spans.append((seg[-1][2] - seg[0][1]) / 1e6)
    out = {p: per[p] / steps for p, _ in PHASES}
    # gloo's staging copies (device <-> host around every collective) do not exist on RCCL, and a visited-set
    # rebuild is a growth event of the run, not a step's work: both shown apart, outside the device total
    stage = sum(v for k, v in unknown.items() if k == '__amd_rocclr_copyBuffer')
    rehash = sum(v for k, v in unknown.items() if k == 'k_rehash')
    out['other'] = (sum(unknown.values()) - stage - rehash) / steps
    out['device total (engine stream)'] = sum(v for k, v in out.items() if not k.startswith('noise'))
    out['gloo staging copies (not on RCCL)'] = stage / steps
    out['visited-set rebuilds'] = rehash / steps
    return out, {k: v / steps for k, v in unknown.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--world', type=int, required=True)
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--out')
    a = ap.parse_args()
    ranks = []
    unk = {}
    allrows = [load(find_trace(os.path.join(a.dir, f'r{r}'))) for r in range(a.world)]
    for r in range(a.world):
        others = [x for q in range(a.world) if q != r for x in allrows[q]]
        ovl = overlap_flags(allrows[r], others) if a.world > 1 else None
        if ovl is not None:
            print(f'rank {r}: {sum(ovl)} of {len(ovl)} kernels overlap another rank\'s (counted at their clean median)')
        t, u = rank_table(allrows[r], a.steps, ovl)
        ranks.append(t)
        for k, v in u.items():
            unk[k] = max(unk.get(k, 0.0), v)
    # robust table: every timed instance capped at 1.5x the median of its kernel's timed instances over all ranks
    inst = defaultdict(list)
    for rows in allrows:
        cut = 'k_mig_digit' if any(r[0] == 'k_mig_digit' for r in rows) else 'k_raw_count'
        ex = [i for i, r in enumerate(rows) if r[0] == cut]
        for name, t0, t1 in rows[ex[-a.steps]:]:
            inst[name].append((t1 - t0) / 1e6)
    cap = {k: 1.5 * sorted(v)[len(v) // 2] for k, v in inst.items()}
    robust = [rank_table(allrows[r], a.steps, None, cap)[0] for r in range(a.world)]
    # per kernel (robust: capped as above), ms per step, mean over ranks: what each phase is made of
    perk = defaultdict(float)
    for rows in allrows:
        cut = 'k_mig_digit' if any(r[0] == 'k_mig_digit' for r in rows) else 'k_raw_count'
        ex = [i for i, r in enumerate(rows) if r[0] == cut]
        for name, t0, t1 in rows[ex[-a.steps]:]:
            perk[name] += min((t1 - t0) / 1e6, cap.get(name, 1e30)) / a.steps / a.world
    keys = list(ranks[0].keys())
    mean = {k: sum(t[k] for t in ranks) / len(ranks) for k in keys}
    worst = {k: max(t[k] for t in ranks) for k in keys}
    rmean = {k: sum(t[k] for t in robust) / len(robust) for k in keys}
    rworst = {k: max(t[k] for t in robust) for k in keys}
    print(f'{"phase":34s} {"mean ms":>9s} {"max ms":>9s} {"robust":>9s} {"rob.max":>9s}')
    for k in keys:
        print(f'{k:34s} {mean[k]:9.3f} {worst[k]:9.3f} {rmean[k]:9.3f} {rworst[k]:9.3f}')
    if unk:
        print('unclassified:', {k: round(v, 3) for k, v in unk.items()})
    print('per kernel (robust ms per step, mean of ranks):',
          ', '.join(f'{k} {v:.3f}' for k, v in sorted(perk.items(), key=lambda kv: -kv[1])[:24]))
    if a.out:
        with open(a.out, 'w') as f:
            json.dump({'world': a.world, 'steps': a.steps, 'mean_ms': mean, 'max_ms': worst, 'per_rank_ms': ranks,
                       'robust_mean_ms': rmean, 'robust_max_ms': rworst, 'robust_per_rank_ms': robust,
                       'unclassified_ms': unk, 'robust_per_kernel_ms': dict(perk)}, f, indent=1)


if __name__ == '__main__':
    main()
