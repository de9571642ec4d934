#!/usr/bin/env python3
"""Oracle-generated goldens for configs the Python reference cannot run here (RAM / time).

The C oracle is pinned bit-exact to the reference's own captures (tests/test_oracle.py: tables,
hashes, successors, scores, MT stream and seeded solves up to W=300k); this script runs it at
larger beam widths and stores the same trace format as tests/golden/make_golden.py (per-turn
n_unique / n_kept / beam digest, solution path, final MT fingerprint).  Test infrastructure only.

    python3 oracle/make_big_golden.py --goal 15 --heur balanced --width 4000000 --seed 0
    python3 oracle/make_big_golden.py --goal 15 --heur efficiency --width 4000000 --seed 0
    python3 oracle/make_big_golden.py --realistic --goal 15 --width 1000000 --seed 0   # C4 (2 players, shuffled)
    python3 oracle/make_big_golden.py --goal 15 --heur efficiency --width 32000000 --seed 0 \
        --lean-log2 32 --spill-dir /tmp                                                   # C5 (W=32M)

C5's width needs the lean knobs to fit a 62 GB host: the visited set (about 2G keys) reserved at
2^32 slots (32 GB, filled to at most 90%), earlier turns' states spilled to an unlinked file, and the
prune's sort scratch sized for the W kept entries only (radix select first).  None of them changes a
result: tests/test_oracle.py runs the W=300k reference solves through the lean path too.
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
    ap.add_argument('--heur', default='balanced')
    ap.add_argument('--realistic', action='store_true',
                    help='MultiPlayerState (src/solver.py:750-860), competitive heuristic, shuffled market')
    ap.add_argument('--players', type=int, default=2)
    ap.add_argument('--width', type=int, required=True)
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--lean-log2', type=int, default=0, help='reserve the visited set at 2^N slots')
    ap.add_argument('--spill-dir', default=None, help='spill earlier turns to a file in this directory')
    ap.add_argument('--out', default=None, help='output path (default tests/golden/<name>.json)')
    a = ap.parse_args()
    if a.realistic:
        return realistic(a)
    random.seed(a.seed)
    st = random.getstate()[1]
    o = oracle_c.OracleSolve(a.goal, use_heuristic=True, heuristic_name=a.heur, beam_width=a.width, mt_state625=st)
    if a.lean_log2 or a.spill_dir:
        o.lean(a.lean_log2, a.spill_dir)
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
        del key
        print(t, turns[-1], 'visited', o.visited_size(), 'maxrss_gb', _maxrss_gb(), flush=True)
    path = o.path()
    out = {'goal': a.goal, 'heuristic': a.heur, 'beam_width': a.width, 'seed': a.seed, 'source': 'oracle_c',
           'moves': len(path) - 1, 'winner_rank': r['winner_rank'],
           'path': [[list(decode(lo, hi)[0]), list(decode(lo, hi)[2]), decode(lo, hi)[3], decode(lo, hi)[4],
                     repr(State.from_packed(lo, hi)), to_signed(state_key(decode(lo, hi)[0], decode(lo, hi)[2]))]
                    for lo, hi in path],
           'turns': turns, 'final_mt': oracle_c.mt_fingerprint(o.mt_state()), 'visited': o.visited_size(),
           'wall_s': round(time.time() - t0, 1)}
    name = f'oracle_g{a.goal}_{a.heur}_w{a.width}_s{a.seed}.json'
    with open(a.out or os.path.join(os.path.dirname(HERE), 'tests', 'golden', name), 'w') as f:
        json.dump(out, f, separators=(',', ':'))
    print('wrote', name, out['moves'], 'moves', out['wall_s'], 's')


def _maxrss_gb():
    import resource
    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 1)


def realistic(a):
    """C4-style golden: the realistic oracle's per-turn digests, the path as packed words, the final MT."""
    import numpy as np
    from splendor_amd.engine_rt import device_tiers
    from splendor_amd.realistic import GameConfig, MultiPlayerState, game_params, pack_state
    cfg = GameConfig(num_players=a.players, target_points=a.goal, gems_per_color={2: 4, 3: 5, 4: 7}[a.players],
                     infinite_resources=False)
    root = MultiPlayerState.newgame(cfg, shuffle_market=True, seed=a.seed)
    tiers0 = device_tiers(root)
    params, tiers = game_params(cfg, tiers0)
    random.seed(a.seed)
    o = oracle_c.OracleRealistic(params, tiers, beam_width=a.width, mt_state625=random.getstate()[1],
                                 root_w=pack_state(root, tiers0))
    turns = []
    t0 = time.time()
    t = 0
    while True:
        ts = time.time()
        r = o.step()
        if r['done']:
            break
        t += 1
        _, _, key = o.turn_arrays(t)
        turns.append({'n_parents': r['n_parents'], 'n_raw': r['n_raw'], 'n_unique': r['n_unique'],
                      'n_kept': r['n_kept'], 'digest': oracle_c.beam_digest(key), 's': round(time.time() - ts, 2)})
        print(t, turns[-1], flush=True)
    path = o.path()
    out = {'goal': a.goal, 'players': a.players, 'shuffle': True, 'beam_width': a.width, 'seed': a.seed,
           'source': 'oracle_c (realistic)', 'moves': len(path) - 1, 'winner_rank': r['winner_rank'],
           'path_words': [[f'{int(x):016x}' for x in row] for row in np.asarray(path)],
           'turns': turns, 'final_mt': oracle_c.mt_fingerprint(o.mt_state()), 'wall_s': round(time.time() - t0, 1)}
    name = f'oracle_realistic_g{a.goal}_p{a.players}_shuf_w{a.width}_s{a.seed}.json'
    with open(os.path.join(os.path.dirname(HERE), 'tests', 'golden', name), 'w') as f:
        json.dump(out, f, separators=(',', ':'))
    print('wrote', name, out['moves'], 'moves', out['wall_s'], 's')


if __name__ == '__main__':
    main()
