"""User-registered Python heuristics (HEURISTICS.md:204-229, src/solver.py:299-305,429) on the product path:
the device expands and dedups, the callable scores next_queue on the host in next_queue order, the device
runs the stable top-k.  Checked against solves captured from the reference with the same callables
registered in its HEURISTICS (tests/golden/make_golden.py custom)."""
import random

import numpy as np
import pytest

import oracle_c
from conftest import golden
from custom_heuristics import CUSTOM
from splendor_amd import _lib as L
from splendor_amd import solver as S
from splendor_amd.engine import BeamEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def registered():
    S.HEURISTICS.update(CUSTOM)
    yield
    for k in CUSTOM:
        S.HEURISTICS.pop(k, None)


def _mt_fp():
    return oracle_c.mt_fingerprint(random.getstate()[1])


@pytest.mark.parametrize('case', range(4))
def test_custom_heuristic_stepwise_golden(case):
    """Every turn's kept beam (digest, sizes) and Python's random state after each prune."""
    g = golden('solves_custom.json')[case]
    h = CUSTOM[g['heuristic']]
    turns = [t for t in g['turns'] if t['n_unique'] > 0]   # the goal turn sorts an empty next_queue
    random.seed(g['seed'])
    eng = BeamEngine(goal_pts=g['goal'], use_heuristic=True, heuristic=L.SB_HEUR_HOST, beam_width=g['beam_width'],
                     mt_state625=random.getstate()[1])
    t = 0
    while True:
        s = eng.step()
        if s['done']:
            break
        kept = eng.prune(S._host_scores(eng, h))
        t += 1
        exp = turns[t - 1]
        assert (s['n_unique'], kept) == (exp['n_unique'], exp['n_kept']), t
        _, _, _, key = eng.read_turn(t)
        assert oracle_c.beam_digest(key) == exp['digest'], f'turn {t}'
        assert _mt_fp() == exp['mt'], f'turn {t}: random state'
    assert t == len(turns)
    assert [S.State.from_packed(*p).hash for p in eng.path()] == [p[5] for p in g['path']]
    assert _mt_fp() == g['final_mt']
    eng.close()


def test_custom_heuristic_solve_golden():
    """State.solve by name, as `-H card_rush` would call it: path and random state as the reference's."""
    for g in golden('solves_custom.json'):
        random.seed(g['seed'])
        path = S.State.newgame().solve(goal_pts=g['goal'], use_heuristic=True, heuristic_name=g['heuristic'],
                                       beam_width=g['beam_width'], verbose=False)
        assert [repr(p) for p in path] == [p[4] for p in g['path']]
        assert [p.hash for p in path] == [p[5] for p in g['path']]
        assert _mt_fp() == g['final_mt']


def test_custom_heuristic_errors():
    S.HEURISTICS['nan'] = lambda st: float('nan')
    S.HEURISTICS['huge'] = lambda st: 2**60 + 1 + st.pts
    try:
        with pytest.raises(L.SplendorBeamError, match='NaN'):
            S.State.newgame().solve(goal_pts=4, use_heuristic=True, heuristic_name='nan', beam_width=50, verbose=False)
        with pytest.raises(TypeError, match='float64'):
            S.State.newgame().solve(goal_pts=4, use_heuristic=True, heuristic_name='huge', beam_width=50,
                                    verbose=False)
    finally:
        S.HEURISTICS.pop('nan')
        S.HEURISTICS.pop('huge')
    # a pending host-scored turn refuses another step, and the score count must match next_queue
    random.seed(0)
    eng = BeamEngine(goal_pts=6, use_heuristic=True, heuristic=L.SB_HEUR_HOST, beam_width=100,
                     mt_state625=random.getstate()[1])
    s = eng.step()
    assert s['n_unique'] > 0 and eng.pending == s['n_unique']
    with pytest.raises(L.SplendorBeamError, match='awaits'):
        eng.step()
    with pytest.raises(L.SplendorBeamError, match='one score per'):
        eng.prune(np.zeros(s['n_unique'] + 1))
    assert eng.prune(np.zeros(s['n_unique'])) == min(100, s['n_unique'])   # all tied: next_queue order
    eng.close()


def test_custom_heuristic_ignored_without_use_heuristic():
    """use_heuristic=False never calls the heuristic (pure BFS, src/solver.py:452-456)."""
    S.HEURISTICS['boom'] = lambda st: 1 / 0
    try:
        path = S.State.newgame().solve(goal_pts=2, use_heuristic=False, heuristic_name='boom', verbose=False)
        assert path[-1].pts >= 2
    finally:
        S.HEURISTICS.pop('boom')


def test_host_scored_topk_arbitrary_keys():
    """sb_prune's top-k on keys of no particular distribution: mixed signs, a 1e-10 tie-break
    jitter (thousands of distinct keys inside one 40-bit prefix run), exact ties and -0.0 == 0.0.  The
    host-scored path sorts on the full key, so the order is the stable sorted(..., reverse=True)."""
    rng = np.random.default_rng(5)
    n = 300_000
    base = rng.choice(np.array([-3.0, -1.0, 0.0, 2.5, 1e6]), n)
    jit = np.where(rng.random(n) < 0.5, rng.random(n) * 1e-10, 0.0)
    s = base + jit
    s[rng.random(n) < 0.01] = -0.0
    for keep in (n, 4096, 77_777):
        out = np.zeros(min(n, keep), np.uint32)
        L.check(L.lib().sb_debug_topk_scores(0, np.ascontiguousarray(s), n, keep, out), 'sb_debug_topk_scores')
        exp = sorted(range(n), key=s.__getitem__, reverse=True)[:keep]
        assert out.tolist() == exp, keep


def _jitter(state):
    return state.pts * 2.0 - sum(state.gems) * 0.5 + (random.random() - 0.5) * 1e-9


def test_host_heuristic_jitter_solve_vs_pyref():
    """A user heuristic with a tiny random tie-break (near-equal, mixed-sign scores) through State.solve,
    against the pure-Python restatement of the reference loop running the same callable."""
    import pyref
    S.HEURISTICS['jitter'] = _jitter
    try:
        random.seed(3)
        path = S.State.newgame().solve(goal_pts=8, use_heuristic=True, heuristic_name='jitter', beam_width=3000,
                                       verbose=False)
        after = random.getstate()
        random.seed(3)
        ps = pyref.PySolve(8, use_heuristic=True, heuristic_name='simple', beam_width=3000, rng=random.Random(0))
        ps.heur = lambda st, _rng: _jitter(st)
        while not ps.step()['done']:
            pass
        assert [p.hash for p in path] == [s.key for s in ps.path()]
        assert random.getstate() == after
    finally:
        S.HEURISTICS.pop('jitter')
