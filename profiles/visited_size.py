#!/usr/bin/env python3
"""Expansion time vs visited-set size on the C3 trajectory (diagnostic; run on the GPU box).
usage: python profiles/visited_size.py 30 31 32   (log2 of the number of 16-byte entries)"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'splendor-rl-gym_amd'))
from splendor_amd.engine import BeamEngine  # noqa: E402

for lg in [int(x) for x in sys.argv[1:]]:
    random.seed(0)
    st = random.getstate()[1]
    eng = BeamEngine(goal_pts=255, use_heuristic=True, heuristic=1, beam_width=4_000_000, mt_state625=st, device=0,
                     timing=True, visited_log2=lg)
    for _ in range(15):
        eng.step()
    eng.sync()
    ex = [eng.turn_times(t)['ms_expand'] for t in range(10, 15)]
    tot = [eng.turn_times(t)['ms_total'] for t in range(10, 15)]
    print(f'visited_log2={lg}: expand turns 10-14 {[round(x, 3) for x in ex]} mean {sum(ex) / 5:.3f} ms; '
          f'step mean {sum(tot) / 5:.3f} ms', flush=True)
    eng.close()
