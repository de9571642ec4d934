"""The C oracle (oracle/csrc/oracle.c) pinned against every golden the reference produced.

CPU-only.  These are the checks that make the oracle trustworthy as the GPU parity checker.
"""
import random

import numpy as np
import pytest

import oracle_c
from conftest import golden, golden_exists
from splendor_amd import codec


def test_take_patterns_match_reference(tables):
    """Pattern tables in distinct_permutations order (src/gems.py:22-37)."""
    L = oracle_c.lib()
    buf = np.zeros(128 * 6, np.int32)
    exp3, exp2 = tables['patterns_take_3_at'], tables['patterns_take_2_at']
    want = {0: exp3['7'] + exp2['8'], 1: exp3['8'] + exp2['8'], 2: exp3['9'] + exp2['9'], 3: exp3['10'] + exp2['10']}
    for b in range(4):
        n = L.oc_patterns(b, buf, 128)
        got = [buf[k * 6:k * 6 + 5].tolist() for k in range(n)]
        assert got == want[b]


def test_takes_and_buys_sample(tables):
    """Takes (ordered) and buys (ordered ids) for sampled gem sets via the successor enumeration."""
    deck = tables['deck']
    for (g, takes), (g2, buys) in zip(tables['takes_sample'], tables['buys_sample']):
        assert g == g2
        if sum(g) > 10:
            continue
        kids = oracle_c.successors((), g, 0, 0)   # no cards, no bonus: key == gems
        got_buys = [k[0][0] for k in kids if k[0]]
        assert got_buys == buys
        got_takes = [list(k[2]) for k in kids if not k[0]]
        assert got_takes == takes
        for c in got_buys:
            assert all(deck[c]['cost'][i] <= g[i] for i in range(5))


def test_hash_vectors(tables):
    for cards, gems, h in tables['hash_vectors']:
        assert oracle_c.state_key(cards, gems) == h


def test_successors(tables):
    for s in tables['successors']:
        cards, bonus, gems, pts, saved, h = s['parent']
        kids = oracle_c.successors(cards, gems, pts, saved)
        exp = [(tuple(c[0]), tuple(c[1]), tuple(c[2]), c[3], c[4], c[5]) for c in s['children']]
        assert kids == exp


@pytest.mark.parametrize('hid,name', [(0, 'simple'), (1, 'balanced'), (2, 'aggressive'), (3, 'efficiency'),
                                      (1, 'competitive')])
def test_scores(tables, hid, name):
    random.seed(11)
    k = random.randint(1, 100)
    for r in tables['heuristic_scores_seed11']:
        lo, hi = codec.encode(r['cards'], r['gems'], r['pts'], r['saved'])
        assert oracle_c.lib().oc_score(lo, hi, hid, k).hex() == r[name]


def test_mt_stream(tables):
    for seed, v in tables['mt'].items():
        out = np.zeros(2000, np.uint32)
        oracle_c.lib().oc_mt_words(np.array(v['state'], np.uint32), out, 2000)
        assert out.tolist() == v['words']
        # randint(1,100) = 1 + (w >> 25), rejecting >= 100
        words = np.zeros(8000, np.uint32)
        oracle_c.lib().oc_mt_words(np.array(v['state'], np.uint32), words, 8000)
        draws = [int(w >> 25) + 1 for w in words if (w >> 25) < 100][:5000]
        assert draws == v['randint']


def _run_oracle(g):
    random.seed(g['seed'])
    st = random.getstate()[1]
    o = oracle_c.OracleSolve(g['goal'], use_heuristic=True, heuristic_name=g['heuristic'],
                             beam_width=g['beam_width'], mt_state625=st)
    turns = [t for t in g['turns'] if t['n_unique'] > 0]
    t = 0
    while True:
        r = o.step()
        if r['done']:
            break
        t += 1
        exp = turns[t - 1]
        assert r['n_unique'] == exp['n_unique']
        _, _, _, key = o.turn_arrays(t)
        assert len(key) == exp['n_kept'] and oracle_c.beam_digest(key) == exp['digest']
    assert t == len(turns)
    keys = [codec.to_signed(oracle_c.lib().oc_state_key(lo, hi)) for lo, hi in o.path()]
    assert keys == [p[5] for p in g['path']]
    assert oracle_c.mt_fingerprint(o.mt_state()) == g['final_mt']
    o.close()


def test_seeded_solves_small():
    for g in golden('solves_small.json'):
        _run_oracle(g)


def test_seeded_solve_c1():
    """Config C1: goal 10 -u -H simple W=300k seed 0 (12 moves)."""
    g = golden('solve_g10_simple_w300000_s0.json')
    assert g['moves'] == 12
    _run_oracle(g)


@pytest.mark.slow
@pytest.mark.parametrize('heur', ['simple', 'balanced', 'aggressive', 'efficiency'])
def test_seeded_solve_goal15_w300k(heur):
    name = f'solve_g15_{heur}_w300000_s0.json'
    if not golden_exists(name):
        pytest.skip('not captured')
    _run_oracle(golden(name))


def test_bfs_paths():
    from splendor_amd.solver import State
    for g in golden('bfs.json'):
        o = oracle_c.OracleSolve(g['goal'], use_heuristic=False, heuristic_name='simple', beam_width=1,
                                 mt_state625=random.getstate()[1])
        o.run()
        assert [repr(State.from_packed(lo, hi)) for lo, hi in o.path()] == [p[4] for p in g['path']]
        o.close()


@pytest.mark.parametrize('seed,n,W,vals', [(0, 5000, 700, 1 << 40), (1, 20000, 19000, 37), (2, 3000, 3000, 5),
                                            (3, 4096, 1, 2), (4, 10000, 2500, 1 << 62), (5, 1, 1, 10), (6, 7, 100, 3)])
def test_oracle_prune_equals_stable_sort_slice(seed, n, W, vals):
    """The oracle's prune (MSB radix select_top of the W-th key, then a stable sort of the candidates: the lean
    path the C5 golden at W=32M came from) equals a full stable descending sort followed by [:W] —
    sorted(next_queue, key=..., reverse=True)[:beam_width] (src/solver.py:452-456) — on random keys with heavy
    ties (few distinct values), full-range keys, W >= n and W = 1."""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, vals, n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15 % vals or 1)
    out = np.zeros(max(min(n, W), 1), np.uint32)
    k = oracle_c.lib().oc_debug_prune(np.ascontiguousarray(key), n, W, out)
    ref = sorted(range(n), key=lambda i: int(key[i]), reverse=True)[:W]   # Python's stable sort, as the reference
    assert k == len(ref) and out[:k].tolist() == ref


def test_oracle_tables_are_its_own():
    """The checker does not share the product's tables: oracle_c / pyref take the deck from the
    fixture captured by importing the reference and restate the state packing (oracle/ref_tables.py); the product's
    deck.py must agree with that capture."""
    import ast
    import os

    import ref_tables
    from conftest import REPO
    from splendor_amd.deck import deck_rows
    for f in ('oracle_c.py', 'pyref.py', 'ref_tables.py'):
        tree = ast.parse(open(os.path.join(REPO, 'oracle', f)).read())
        mods = {n.module for n in ast.walk(tree) if isinstance(n, ast.ImportFrom) and n.module}
        mods |= {a.name for n in ast.walk(tree) if isinstance(n, ast.Import) for a in n.names}
        assert not any(m.startswith('splendor_amd') for m in mods), (f, mods)
    assert ref_tables.deck_rows() == list(deck_rows())
