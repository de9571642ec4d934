"""The pure-Python restatement (oracle/pyref.py, bench.py's reference-style CPU leg) pinned against the
reference's captures, as the C oracle is in test_oracle.py.  CPU-only."""
import random

import pytest

import pyref
from conftest import golden


def test_successors_match_reference(tables):
    for s in tables['successors']:
        cards, bonus, gems, pts, saved, h = s['parent']
        p = pyref.PState(tuple(cards), tuple(bonus), tuple(gems), pts, saved)
        assert p.key == h
        got = [(c.cards, c.bonus, c.gems, c.pts, c.saved, c.key) for c in p.children()]
        exp = [(tuple(c[0]), tuple(c[1]), tuple(c[2]), c[3], c[4], c[5]) for c in s['children']]
        assert got == exp


def test_hash_vectors(tables):
    for cards, gems, h in tables['hash_vectors'][:500]:
        assert pyref.PState(tuple(cards), (0,) * 5, tuple(gems), 0, 0).key == h


@pytest.mark.parametrize('name', ['simple', 'balanced', 'aggressive', 'efficiency', 'competitive'])
def test_scores(tables, name):
    for r in tables['heuristic_scores_seed11']:
        bonus = [0] * 5
        for c in r['cards']:
            bonus[pyref.DECK[c][2]] += 1
        s = pyref.PState(tuple(r['cards']), tuple(bonus), tuple(r['gems']), r['pts'], r['saved'])
        rng = random.Random(11)
        assert pyref.HEURISTICS[name](s, rng).hex() == r[name]


def _run(g):
    random.seed(g['seed'])
    o = pyref.PySolve(g['goal'], use_heuristic=True, heuristic_name=g['heuristic'], beam_width=g['beam_width'],
                      mt_state625=random.getstate()[1])
    turns = [t for t in g['turns'] if t['n_unique'] > 0]
    t = 0
    while True:
        r = o.step()
        if r['done']:
            break
        t += 1
        exp = turns[t - 1]
        assert r['n_unique'] == exp['n_unique'] and r['n_kept'] == exp['n_kept']
        assert pyref.beam_digest(o.keys(t)) == exp['digest']
    assert t == len(turns)
    assert [s.key for s in o.path()] == [p[5] for p in g['path']]
    import oracle_c
    assert oracle_c.mt_fingerprint(o.mt_state()) == g['final_mt']


def test_seeded_solves_small():
    """Goal 6 at W=1k, all heuristics incl. the unknown-name fallback (reference captures)."""
    for g in golden('solves_small.json'):
        if g['goal'] == 6 and g['beam_width'] == 1000:
            _run(g)


def test_seeded_solve_goal10_w1k():
    for g in golden('solves_small.json'):
        if g['goal'] == 10 and g['beam_width'] == 1000 and g['seed'] == 0 and g['heuristic'] in ('simple', 'efficiency'):
            _run(g)


def test_from_oracle_sample_is_the_turns_prefix():
    """bench.py's CPU baseline: the pure-Python step on the first k parents of the oracle's newest beam (same
    config and MT state), with a trail of that beam's keys."""
    import numpy as np
    import oracle_c
    random.seed(0)
    o = oracle_c.OracleSolve(255, use_heuristic=True, heuristic_name='balanced', beam_width=2000,
                             mt_state625=random.getstate()[1])
    for _ in range(5):
        o.step()
    lo, hi, _, key = o.turn_arrays(o.nturns() - 1)
    ps = pyref.from_oracle(o, 255, 'balanced', 2000, sample=50)
    assert [s.key for s in ps.turns[0][0]] == np.asarray(key[:50]).view(np.int64).tolist()
    assert len(ps.trail) == len(set(np.asarray(key).view(np.int64).tolist()))
    r = ps.step()
    assert r['n_parents'] == 50 and r['n_raw'] > 0 and 0 < r['n_kept'] <= 2000
    o.close()
