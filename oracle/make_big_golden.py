#!/usr/bin/env python3
"""Oracle-generated goldens for configs the Python reference cannot run here (RAM / time).

The C oracle is pinned bit-exact to the reference's own captures (tests/test_oracle.py: tables,
hashes, successors, scores, MT stream and seeded solves up to W=300k); this script runs it at
larger beam widths and stores the same trace format as tests/golden/make_golden.py (per-turn
n_unique / n_kept / beam digest, solution path, final MT fingerprint).  Test infrastructure only.

    python3 oracle/make_big_golden.py --goal 15 --heur balanced --width 4000000 --seed 0
"""
import argparse
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle_c  # noqa: E402
from splendor_amd.codec import decode, state_key, to_signed  # noqa: E402
from splendor_amd.solver import State  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--goal', type=int, required=True)
    ap.add_argument('--heur', required=True)
    ap.add_argument('--width', type=int, required=True)
    ap.add_argument('--seed', type=int, default=0)
    a = ap.parse_args()
    random.seed(a.seed)
    st = random.getstate()[1]
    o = oracle_c.OracleSolve(a.goal, use_heuristic=True, heuristic_name=a.heur, beam_width=a.width, mt_state625=st)
    turns = []
    t0 = time.time()
    t = 0
    while True:
        ts = time.time()
        r = o.step()
        if r['done']:
            break
        t += 1
        _, _, _, key = o.turn_arrays(t)
        turns.append({'n_parents': r['n_parents'], 'n_raw': r['n_raw'], 'n_unique': r['n_unique'],
                      'n_kept': r['n_kept'], 'digest': oracle_c.beam_digest(key), 's': round(time.time() - ts, 2)})
        print(t, turns[-1], flush=True)
    path = o.path()
    out = {'goal': a.goal, 'heuristic': a.heur, 'beam_width': a.width, 'seed': a.seed, 'source': 'oracle_c',
           'moves': len(path) - 1, 'winner_rank': r['winner_rank'],
           'path': [[list(decode(lo, hi)[0]), list(decode(lo, hi)[2]), decode(lo, hi)[3], decode(lo, hi)[4],
                     repr(State.from_packed(lo, hi)), to_signed(state_key(decode(lo, hi)[0], decode(lo, hi)[2]))]
                    for lo, hi in path],
           'turns': turns, 'final_mt': oracle_c.mt_fingerprint(o.mt_state()), 'visited': o.visited_size(),
           'wall_s': round(time.time() - t0, 1)}
    name = f'oracle_g{a.goal}_{a.heur}_w{a.width}_s{a.seed}.json'
    with open(os.path.join(os.path.dirname(HERE), 'tests', 'golden', name), 'w') as f:
        json.dump(out, f, separators=(',', ':'))
    print('wrote', name, out['moves'], 'moves', out['wall_s'], 's')


if __name__ == '__main__':
    main()
