#!/usr/bin/env python3
"""The bias of bench.py's pure-Python CPU baseline sample, measured once on CPU.

The baseline times the reference's step (oracle/pyref.py) on the first 100k parents of C3's first timed turn (W=4M,
turn 9) with a trail holding only that beam's keys: a child first seen in an older turn is treated as new — scored,
appended to next_queue and sorted.  Here the same sample step runs, and its new children are then looked up in the C
oracle's full trail (every key visited through turn 8, oc_visited_keys): those found there are the ones the reference
would have dropped.  Reports both counts and the timing with each trail kind (the exact trail is a Python set of the
sample's parents' children that are in the full trail plus the beam: it changes only the membership answers).
    python3 profiles/cpu_baseline_bias.py [--width 4000000] [--turn 9] [--sample 100000] [--out FILE]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, 'oracle'), os.path.join(HERE, 'splendor-rl-gym_amd')]


def main():
    import oracle_c
    import pyref
    ap = argparse.ArgumentParser()
    ap.add_argument('--width', type=int, default=4_000_000)
    ap.add_argument('--turn', type=int, default=9)
    ap.add_argument('--sample', type=int, default=100_000)
    ap.add_argument('--heuristic', default='balanced')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    random.seed(0)
    o = oracle_c.OracleSolve(255, use_heuristic=True, heuristic_name=a.heuristic, beam_width=a.width,
                             mt_state625=random.getstate()[1])
    t0 = time.perf_counter()
    for _ in range(a.turn):
        o.step()
    setup = time.perf_counter() - t0
    full = np.sort(o.visited_keys().view(np.int64))
    # as bench.py times it: trail = the newest beam's keys
    ps = pyref.from_oracle(o, 255, a.heuristic, a.width, sample=a.sample)
    t0 = time.perf_counter()
    r = ps.step()
    dt_beam = time.perf_counter() - t0
    # the sample's next_queue before the prune: rerun the expansion to list the new children (no timing)
    ps2 = pyref.from_oracle(o, 255, a.heuristic, a.width, sample=a.sample)
    queue, _ = ps2.turns[-1]
    trail = ps2.trail
    new = []
    for s in queue:
        for ch in s.children():
            if ch.key in trail:
                continue
            trail.add(ch.key)
            new.append(ch.key)
    new = np.array(new, dtype=np.int64)
    i = np.searchsorted(full, new)
    found = (i < len(full)) & (full[np.minimum(i, len(full) - 1)] == new)
    # the same step with the exact answers: a trail of the beam's keys plus the sample's children that the full trail
    # holds (what the reference's trail would answer for these children)
    ps3 = pyref.from_oracle(o, 255, a.heuristic, a.width, sample=a.sample)
    ps3.trail |= set(new[found].tolist())
    t0 = time.perf_counter()
    r3 = ps3.step()
    dt_exact = time.perf_counter() - t0
    o.close()
    out = {'width': a.width, 'turn': a.turn, 'sample_parents': r['n_parents'], 'raw_children': r['n_raw'],
           'new_with_beam_trail': int(r['n_unique']), 'of_them_in_older_turns': int(found.sum()),
           'new_exact': int(r3['n_unique']),
           'states_per_s_beam_trail': round(r['n_parents'] / dt_beam, 1),
           'states_per_s_exact_trail': round(r3['n_parents'] / dt_exact, 1),
           'setup_s': round(setup, 1), 'host': os.uname().nodename, 'python': sys.version.split()[0]}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
