#!/usr/bin/env python3
"""Where the next beam comes from (the kept records of the key-owner protocol leave rank 0): for each
saturated turn of a seeded C oracle solve, the share of the kept states whose parent lies in each block of the
parent ranking, and the largest per-rank share if the parents were dealt to G ranks in P x G interleaved blocks
(P = 1: contiguous rank ranges, as the sharded step holds them).  python3 profiles/analysis/kept_dist.py W heuristic"""
import random, sys, numpy as np
sys.path.insert(0, 'oracle'); sys.path.insert(0, 'splendor-rl-gym_amd')
import oracle_c
W = int(sys.argv[1]); heur = sys.argv[2]
random.seed(0)
o = oracle_c.OracleSolve(15, use_heuristic=True, heuristic_name=heur, beam_width=W, mt_state625=random.getstate()[1])
tr = o.run()
n = o.nturns()
for t in range(1, n):
    lo, hi, par, key = o.turn_arrays(t)
    npar = len(o.turn_arrays(t - 1)[0])
    if npar < W: continue
    h = np.bincount(par.astype(np.int64) * 128 // npar, minlength=128)
    f = h / h.sum()
    for G, P in ((8, 1), (8, 4), (8, 16)):
        nb = G * P
        blk = np.bincount(par.astype(np.int64) * nb // npar, minlength=nb) / len(par)
        per_rank = np.array([blk[r::G].sum() for r in range(G)])
        print(f'turn {t} G={G} P={P}: max rank share {per_rank.max():.3f} (balanced {1/G:.3f}); rank shares {np.round(per_rank, 3).tolist()}')
    print(f'turn {t}: top 1/128 of parents -> {f[0]:.3f} of kept, top 1/32 -> {f[:4].sum():.3f}, top 1/8 -> {f[:16].sum():.3f}')
