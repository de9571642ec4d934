#!/usr/bin/env python3
"""How many kept children travel per (parent, destination) group on the rebalance's wire (grouped kept records,
sbd_pack_kept_grouped): for each saturated turn of a seeded C oracle solve at world G, per source rank (contiguous
parent ranges) the kept children it sends to other ranks (destinations: contiguous ranges of the new beam), the
distinct (parent, destination) pairs among them, and the bytes grouped (20 per group + 2 per child) against the
20-byte records (20 per child).  python3 profiles/analysis/kept_groups.py W heuristic [G]"""
import random, sys, numpy as np
sys.path.insert(0, 'oracle'); sys.path.insert(0, 'splendor-rl-gym_amd')
import oracle_c
W = int(sys.argv[1]); heur = sys.argv[2]; G = int(sys.argv[3]) if len(sys.argv) > 3 else 8
random.seed(0)
o = oracle_c.OracleSolve(15, use_heuristic=True, heuristic_name=heur, beam_width=W, mt_state625=random.getstate()[1])
o.run()
for t in range(1, o.nturns()):
    lo, hi, par, key = o.turn_arrays(t)
    npar = len(o.turn_arrays(t - 1)[0])
    if npar < W:
        continue
    m = len(par)
    src = par.astype(np.int64) * G // npar
    dst = np.arange(m, dtype=np.int64) * G // m
    rows = []
    for s in range(G):
        sel = (src == s) & (dst != s)
        nrec = int(sel.sum())
        pairs = np.unique(par[sel].astype(np.int64) * G + dst[sel]).size
        rows.append((s, nrec, pairs, 20 * nrec, 20 * pairs + 2 * nrec))
    worst = max(rows, key=lambda r: r[3])
    print(f'turn {t}: busiest source {worst[0]}: {worst[1]} remote kept children in {worst[2]} groups '
          f'({worst[1] / max(worst[2], 1):.2f} per group): {worst[4] / max(worst[3], 1):.3f} of the 20-byte bytes; '
          f'all sources: {sum(r[4] for r in rows) / max(sum(r[3] for r in rows), 1):.3f}')
