#!/usr/bin/env python3
"""Golden-vector capture from the reference (run ONLY in the survey/build container).

This script imports IamJasonBian/Splendor-RL-Gym from a *writable copy* of the
reference (``REF_PATH``, default ``/tmp/refcopy``) with the offline
``more_itertools`` shim on ``PYTHONPATH`` (recipe: SURVEY.md §8c), runs the
reference code and writes small JSON fixtures (inputs + expected outputs) next
to this file.  Nothing under ``tests/`` imports the reference at test time;
the GPU box never sees it.  The fixtures are data, not reference source.

Usage (from the repo root)::

    mkdir -p /tmp/oracle_shim && ln -s /opt/conda/lib/python3.9/site-packages/more_itertools /tmp/oracle_shim/
    cp -r /root/reference /tmp/refcopy
    PYTHONPATH=/tmp/oracle_shim:/tmp/refcopy python3 tests/golden/make_golden.py tables
    PYTHONPATH=... python3 tests/golden/make_golden.py solve --goal 10 --heur simple --width 300000 --seed 0

The reference's shipped buys.pickle is never unpickled: delete it from the copy first
(``rm /tmp/refcopy/buys.pickle``), so the reference generates and pickles its own table.

Digest convention (shared with ``oracle/`` and the engine): the digest of a beam
is ``sha256(b''.join(struct.pack('<q', hash(s)) for s in beam)).hexdigest()[:16]``.
"""
import argparse
import hashlib
import json
import os
import random
import struct
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REF_PATH = os.environ.get('REF_PATH', '/tmp/refcopy')
if REF_PATH not in sys.path:
    sys.path.insert(0, REF_PATH)


def _digest(states):
    return hashlib.sha256(b''.join(struct.pack('<q', hash(s)) for s in states)).hexdigest()[:16]


def _mt_fingerprint():
    st = random.getstate()
    return {'pos': st[1][-1],
            'sha': hashlib.sha256(struct.pack('<625I', *st[1])).hexdigest()[:16]}


def _dump(name, obj):
    path = os.path.join(HERE, name)
    with open(path, 'w') as f:
        json.dump(obj, f, separators=(',', ':'))
    print('wrote', path, os.path.getsize(path), 'bytes')


def cmd_tables(_args):
    from src import gems as G
    from src.buys import possible_buys
    from src.cardparser import get_deck
    from src.solver import State

    deck = get_deck()
    out = {}
    out['deck'] = [{'cost': list(c.cost), 'pt': c.pt, 'color': c.bonus.value,
                    'str_id': c.str_id} for c in deck]
    out['patterns_take_3_at'] = {k: [list(p) for p in v] for k, v in G.patterns_take_3_at.items()}
    out['patterns_take_2_at'] = {k: [list(p) for p in v] for k, v in G.patterns_take_2_at.items()}

    takes = G.get_takes()
    h = hashlib.sha256()
    for g in G.all_gem_sets:
        h.update(repr(takes[g]).encode())
    out['takes_sha256'] = h.hexdigest()
    rng = random.Random(1234)
    sample = [tuple(rng.randrange(8) for _ in range(5)) for _ in range(400)]
    sample += [(0, 0, 0, 0, 0), (6, 0, 0, 0, 0), (7, 7, 7, 7, 7), (3, 3, 2, 1, 1), (2, 2, 2, 2, 2)]
    out['takes_sample'] = [[list(g), [list(t) for t in takes[g]]] for g in sample]

    buys = possible_buys()
    h = hashlib.sha256()
    for g in G.all_gem_sets:
        h.update(repr(buys[g]).encode())
    out['buys_sha256'] = h.hexdigest()
    out['buys_sample'] = [[list(g), list(buys[g])] for g in sample]

    # pow tables: exact doubles (hex) of float(x) ** e for the exponents the heuristics use
    exps = [0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 1.2, 2.0, 2.5, 2.8, 3.2]
    out['pow_tables'] = {repr(e): [float(x ** e).hex() for x in range(256)] for e in exps}
    out['noise_table'] = [float(k * 0.01).hex() for k in range(1, 101)]

    # MT19937 / randint stream model
    mt = {}
    for s in (0, 1, 12345):
        random.seed(s)
        st = random.getstate()
        words = [random.getrandbits(32) for _ in range(2000)]
        random.seed(s)
        draws = [random.randint(1, 100) for _ in range(5000)]
        after = _mt_fingerprint()
        mt[str(s)] = {'state': list(st[1]), 'words': words, 'randint': draws, 'after_randint': after}
    out['mt'] = mt

    # CPython tuple hash of (cards, gems)
    rng = random.Random(99)
    hv = []
    for _ in range(3000):
        n = rng.randrange(0, 25)
        cards = tuple(sorted(rng.sample(range(90), n)))
        gems = tuple(rng.randrange(8) for _ in range(5))
        hv.append([list(cards), list(gems), hash((cards, gems))])
    hv.append([[], [0, 0, 0, 0, 0], hash(((), (0, 0, 0, 0, 0)))])
    out['hash_vectors'] = hv

    # Ordered successor lists of reachable states (random walks from the root)
    rng = random.Random(7)
    succ = []
    seen = set()
    for walk in range(60):
        st = State.newgame()
        for depth in range(rng.randrange(1, 22)):
            kids = list(st)
            if not kids:
                break
            st = kids[rng.randrange(len(kids))]
            if depth % 3 == 0 and st.hash not in seen:
                seen.add(st.hash)
                kids2 = list(st)
                succ.append({'parent': [list(st.cards), list(st.bonus), list(st.gems), st.pts, st.saved, st.hash],
                             'children': [[list(c.cards), list(c.bonus), list(c.gems), c.pts, c.saved, c.hash]
                                          for c in kids2]})
    out['successors'] = succ

    # heuristic scores without noise pinned through the exact noise draw: evaluate with a fixed seed
    import src.solver as S
    hs = []
    rng = random.Random(5)
    for _ in range(300):
        cards = tuple(sorted(rng.sample(range(90), rng.randrange(0, 20))))
        bonus = [0] * 5
        pts = 0
        for c in cards:
            bonus[deck[c].bonus.value] += 1
            pts += deck[c].pt
        st = State(cards, tuple(bonus), tuple(rng.randrange(8) for _ in range(5)), pts, rng.randrange(0, 40))
        row = {'cards': list(cards), 'gems': list(st.gems), 'pts': pts, 'saved': st.saved, 'bonus': bonus}
        for name in ('simple', 'balanced', 'aggressive', 'efficiency', 'competitive'):
            random.seed(11)
            row[name] = S.HEURISTICS[name](st).hex()
        hs.append(row)
    out['heuristic_scores_seed11'] = hs

    # repr of states
    out['repr'] = [[list(s['parent'][0]), list(s['parent'][2]),
                    repr(State(tuple(s['parent'][0]), tuple(s['parent'][1]), tuple(s['parent'][2]),
                               s['parent'][3], s['parent'][4]))] for s in succ[:50]]
    _dump('tables.json', out)


def _run_speedrun(goal, heur, width, seed, use_heuristic=True):
    import src.solver as S
    trace = []
    real_sorted = sorted

    def traced_sorted(seq, key=None, reverse=False):
        t0 = time.time()
        res = real_sorted(seq, key=key, reverse=reverse)
        kept = res[:width]
        trace.append({'n_unique': len(seq), 'n_kept': len(kept), 'digest': _digest(kept),
                      'head': repr(kept[0]) if kept else None,
                      'head_pts': kept[0].pts if kept else None,
                      'mt': _mt_fingerprint(), 'sort_s': round(time.time() - t0, 3)})
        return res

    S.sorted = traced_sorted
    try:
        random.seed(seed)
        t0 = time.time()
        sol = S.State.newgame().solve(goal_pts=goal, use_heuristic=use_heuristic, heuristic_name=heur,
                                      beam_width=width, verbose=False)
        wall = time.time() - t0
    finally:
        del S.sorted
    return {'goal': goal, 'heuristic': heur, 'beam_width': width, 'seed': seed,
            'use_heuristic': use_heuristic, 'moves': len(sol) - 1,
            'path': [[list(s.cards), list(s.gems), s.pts, s.saved, repr(s), s.hash] for s in sol],
            'turns': trace, 'final_mt': _mt_fingerprint(), 'wall_s': round(wall, 2)}


def cmd_solve(args):
    res = _run_speedrun(args.goal, args.heur, args.width, args.seed)
    _dump(f'solve_g{args.goal}_{args.heur}_w{args.width}_s{args.seed}.json', res)


def cmd_solves_small(_args):
    out = []
    for goal in (6, 10):
        for heur in ('simple', 'balanced', 'aggressive', 'efficiency', 'competitive', 'nonexistent'):
            for width in (1000, 10000):
                for seed in (0, 1):
                    if goal == 10 and width == 10000 and seed == 1:
                        continue
                    r = _run_speedrun(goal, heur, width, seed)
                    print(goal, heur, width, seed, r['moves'], r['wall_s'])
                    out.append(r)
    _dump('solves_small.json', out)


def cmd_bfs(_args):
    import src.solver as S
    out = []
    for goal in (1, 2, 3, 4):
        sol = S.State.newgame().solve(goal_pts=goal, verbose=False)
        out.append({'goal': goal, 'path': [[list(s.cards), list(s.gems), s.pts, s.saved, repr(s), s.hash]
                                           for s in sol]})
    # BFS queue sizes per turn (first turns only) via a standalone replay of the loop counts
    _dump('bfs.json', out)


def cmd_custom(_args):
    """Seeded solves with user-registered heuristics (tests/custom_heuristics.py) added to HEURISTICS."""
    import src.solver as S
    sys.path.insert(0, os.path.dirname(HERE))
    from custom_heuristics import CASES, CUSTOM
    S.HEURISTICS.update(CUSTOM)
    out = []
    for goal, name, width, seed in CASES:
        r = _run_speedrun(goal, name, width, seed)
        print(goal, name, width, seed, r['moves'], r['wall_s'])
        out.append(r)
    _dump('solves_custom.json', out)


def cmd_verbose(_args):
    """stdout of the reference CLI (splendor_fastest_win.py) without -q, random.seed(0), each in a fresh process
    (the reference's buys-table messages are whatever its first get_buys() prints in that process)."""
    import subprocess
    out = []
    code = ('import random, sys; random.seed(0); sys.argv = ["splendor_fastest_win.py"] + sys.argv[1:]; '
            'import splendor_fastest_win as F; F.cli()')
    for argv in (['6', '-u', '-w', '1000'], ['4'], ['7', '-u', '-H', 'balanced', '-w', '500', '-r'],
                 ['6', '--realistic', '-w', '3000'], ['5', '--realistic', '--players', '3', '-w', '400']):
        r = subprocess.run([sys.executable, '-c', code, *argv], capture_output=True, text=True, cwd=REF_PATH,
                           check=True)
        out.append({'argv': argv, 'seed': 0, 'stdout': r.stdout})
        print(argv, len(r.stdout.splitlines()), 'lines')
    _dump('cli_verbose.json', out)


def _mp_key(st):
    return st.hash


def _run_realistic(goal, width, seed, shuffle, players=2, infinite=False):
    import src.solver as S
    trace = []
    real_sorted = sorted

    def traced_sorted(seq, key=None, reverse=False):
        res = real_sorted(seq, key=key, reverse=reverse)
        if key is None:          # card-tuple sorts inside MultiPlayerState.__iter__ (src/solver.py:590)
            return res
        kept = res[:width]
        trace.append({'n_unique': len(seq), 'n_kept': len(kept), 'digest': _digest(kept),
                      'mt': _mt_fingerprint()})
        return res

    gems_per_color = {2: 4, 3: 5, 4: 7}.get(players, 4)
    config = S.GameConfig(num_players=players, target_points=goal, gems_per_color=gems_per_color,
                          infinite_resources=infinite)
    S.sorted = traced_sorted
    try:
        g = S.MultiPlayerState.newgame(config=config, shuffle_market=shuffle, seed=seed if shuffle else None)
        random.seed(seed)
        t0 = time.time()
        sol = g.solve(use_heuristic=True, heuristic_name='competitive', beam_width=width, verbose=False)
        wall = time.time() - t0
    finally:
        del S.sorted
    last = sol[-1]
    m = g.market
    return {'goal': goal, 'beam_width': width, 'seed': seed, 'shuffle': shuffle, 'players': players,
            'infinite': infinite,
            'market': {'t1': list(m.tier1_visible) + list(m.tier1_deck),
                       't2': list(m.tier2_visible) + list(m.tier2_deck),
                       't3': list(m.tier3_visible) + list(m.tier3_deck)},
            'moves': last.turn_number, 'winner': last.get_winner(),
            'final': [[p.player_id, list(p.cards), list(p.bonus), list(p.gems), p.pts, p.saved]
                      for p in last.players],
            'path': [{'hash': s.hash, 'repr': repr(s), 'cur': s.current_player, 'turn': s.turn_number,
                      'frt': s.final_round_triggered, 'frp': s.final_round_player,
                      'pool': list(s.gem_pool.available), 'visible': list(s.market.all_visible_cards()),
                      'players': [[p.player_id, list(p.cards), list(p.gems), p.pts, p.saved] for p in s.players]}
                     for s in sol],
            'turns': trace, 'final_mt': _mt_fingerprint(), 'wall_s': round(wall, 2)}


def cmd_realistic(args):
    res = _run_realistic(args.goal, args.width, args.seed, args.shuffle, args.players)
    tag = 'shuf' if args.shuffle else 'fixed'
    _dump(f'realistic_g{args.goal}_p{args.players}_{tag}_w{args.width}_s{args.seed}.json', res)


def _competitive_heuristic():
    """The reference's multi_competitive_heuristic is a closure inside MultiPlayerState.solve
    (src/solver.py:778-812); rebuild it from its code object (no reference file is modified)."""
    import types
    import src.solver as S
    for c in S.MultiPlayerState.solve.__code__.co_consts:
        if isinstance(c, types.CodeType) and c.co_name == 'multi_competitive_heuristic':
            return types.FunctionType(c, S.__dict__)
    raise RuntimeError('closure not found')


def _enc_mp(s):
    return {'hash': s.hash, 'cur': s.current_player, 'turn': s.turn_number,
            'frt': s.final_round_triggered, 'frp': s.final_round_player,
            'pool': list(s.gem_pool.available),
            'vis': [list(s.market.tier1_visible), list(s.market.tier2_visible), list(s.market.tier3_visible)],
            'decklen': [len(s.market.tier1_deck), len(s.market.tier2_deck), len(s.market.tier3_deck)],
            'players': [[p.player_id, list(p.cards), list(p.bonus), list(p.gems), p.pts, p.saved] for p in s.players],
            'game_over': s.is_game_over()}


def cmd_realistic_succ(args, infinite=False, walks=60, name='realistic_succ.json'):
    """Ordered successor lists + hashes + competitive scores for realistic states (buy-biased walks)."""
    import src.solver as S
    heur = _competitive_heuristic()
    out = []
    rng = random.Random(3 if not infinite else 13)
    for players in (2, 3, 4):
        gpc = {2: 4, 3: 5, 4: 7}[players]
        for walk in range(walks):
            target = rng.choice((3, 6, 15))
            cfg = S.GameConfig(num_players=players, target_points=target, gems_per_color=gpc,
                               infinite_resources=infinite)
            st = S.MultiPlayerState.newgame(cfg, shuffle_market=bool(walk % 2), seed=walk)
            m = st.market
            depth = rng.randrange(1, 60)
            for _ in range(depth):
                kids = list(st)
                if not kids:
                    break
                buys = [k for k in kids if sum(len(p.cards) for p in k.players) > sum(len(p.cards) for p in st.players)]
                st = rng.choice(buys) if buys and rng.random() < 0.7 else rng.choice(kids)
                if st.is_game_over():
                    break
            kids = list(st)
            scores = []
            for k in kids:
                random.seed(17)
                scores.append(heur(k).hex())
            out.append({'players': players, 'target': target, 'shuffle': bool(walk % 2), 'seed': walk,
                        'infinite': infinite,
                        'market0': {'t1': list(m.tier1_visible) + list(m.tier1_deck),
                                    't2': list(m.tier2_visible) + list(m.tier2_deck),
                                    't3': list(m.tier3_visible) + list(m.tier3_deck)},
                        'state': _enc_mp(st), 'children': [_enc_mp(k) for k in kids], 'scores_seed17': scores,
                        'winner': st.get_winner()})
    _dump(name, out)


def cmd_realistic_inf_succ(args):
    """The same captures with infinite_resources=True (takes = the speedrun take table, src/solver.py:635-659)."""
    cmd_realistic_succ(args, infinite=True, walks=20, name='realistic_inf_succ.json')


def cmd_realistic_inf_small(_args):
    out = []
    for goal, width, seed, shuffle, players in [(5, 300, 1, False, 2), (6, 1000, 2, True, 2), (8, 2000, 3, True, 2),
                                                  (4, 200, 4, False, 3), (3, 100, 6, True, 4)]:
        r = _run_realistic(goal, width, seed, shuffle, players, infinite=True)
        print(goal, width, seed, shuffle, players, r['moves'], r['wall_s'])
        out.append(r)
    _dump('realistic_inf_small.json', out)


def cmd_realistic_small(_args):
    out = []
    for goal, width, seed, shuffle, players in [(5, 500, 1, False, 2), (6, 300, 2, True, 2), (8, 2000, 3, True, 2),
                                                  (4, 100, 4, False, 3), (6, 1000, 5, True, 2), (3, 50, 6, True, 4)]:
        r = _run_realistic(goal, width, seed, shuffle, players)
        print(goal, width, seed, shuffle, players, r['moves'], r['wall_s'])
        out.append(r)
    _dump('realistic_small.json', out)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest='cmd', required=True)
    sub.add_parser('tables')
    sub.add_parser('solves_small')
    sub.add_parser('bfs')
    sub.add_parser('realistic_succ')
    sub.add_parser('realistic_small')
    sub.add_parser('realistic_inf_succ')
    sub.add_parser('realistic_inf_small')
    sub.add_parser('custom')
    sub.add_parser('verbose')
    p = sub.add_parser('solve')
    p.add_argument('--goal', type=int, required=True)
    p.add_argument('--heur', required=True)
    p.add_argument('--width', type=int, required=True)
    p.add_argument('--seed', type=int, default=0)
    p = sub.add_parser('realistic')
    p.add_argument('--goal', type=int, required=True)
    p.add_argument('--width', type=int, required=True)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--players', type=int, default=2)
    p.add_argument('--shuffle', action='store_true')
    args = ap.parse_args()
    {'tables': cmd_tables, 'solve': cmd_solve, 'solves_small': cmd_solves_small, 'bfs': cmd_bfs,
     'realistic': cmd_realistic, 'realistic_succ': cmd_realistic_succ, 'custom': cmd_custom,
     'verbose': cmd_verbose,
     'realistic_small': cmd_realistic_small, 'realistic_inf_succ': cmd_realistic_inf_succ,
     'realistic_inf_small': cmd_realistic_inf_small}[args.cmd](args)


if __name__ == '__main__':
    main()
