"""Realistic mode on the GPU (sbr_*): per-turn beams, paths and MT state vs the reference's captures and
the realistic C oracle."""
import random

import numpy as np
import pytest

import oracle_c
from conftest import golden
from splendor_amd.engine_rt import RealisticEngine
from splendor_amd.realistic import GameConfig, MultiPlayerState, game_params, pack_state

pytestmark = pytest.mark.gpu


def _root(g):
    cfg = GameConfig(num_players=g['players'], target_points=g['goal'],
                     gems_per_color={2: 4, 3: 5, 4: 7}[g['players']], infinite_resources=g.get('infinite', False))
    return MultiPlayerState.newgame(cfg, shuffle_market=g['shuffle'], seed=g['seed'] if g['shuffle'] else None)


def _check(g):
    root = _root(g)
    random.seed(g['seed'])
    eng = RealisticEngine(root, beam_width=g['beam_width'], mt_state625=random.getstate()[1])
    turns = [t for t in g['turns'] if t['n_unique'] > 0]
    t = 0
    while True:
        s = eng.step()
        if s['done']:
            break
        t += 1
        exp = turns[t - 1]
        _, _, key = eng.read_turn(t)
        assert s['n_unique'] == exp['n_unique'] and len(key) == exp['n_kept'], t
        assert oracle_c.beam_digest(key) == exp['digest'], f'turn {t}'
    assert t == len(turns)
    path = eng.path()
    assert [p.hash for p in path] == [p['hash'] for p in g['path']]
    assert path[-1].turn_number == g['moves'] and path[-1].get_winner() == g['winner']
    assert oracle_c.mt_fingerprint(eng.mt_state()) == g['final_mt']
    eng.close()


def test_realistic_small_golden():
    for g in golden('realistic_small.json'):
        _check(g)


def test_realistic_infinite_small_golden():
    """infinite_resources=True (speedrun takes, the pool only grows, src/solver.py:635-659)."""
    for g in golden('realistic_inf_small.json'):
        _check(g)


def test_realistic_readme_example_golden():
    _check(golden('realistic_g6_p2_fixed_w3000_s0.json'))


def test_realistic_goal15_w20k_golden():
    _check(golden('realistic_g15_p2_shuf_w20000_s0.json'))


def test_realistic_vs_oracle_stepwise():
    for goal, width, seed, shuffle, players, inf in [(7, 4000, 11, True, 2, False), (5, 800, 12, False, 3, False),
                                                     (4, 300, 13, True, 4, False), (9, 20000, 14, True, 2, True),
                                                     (6, 2000, 15, False, 3, True)]:
        g = {'players': players, 'goal': goal, 'shuffle': shuffle, 'seed': seed, 'infinite': inf}
        root = _root(g)
        random.seed(seed)
        st = random.getstate()[1]
        eng = RealisticEngine(root, beam_width=width, mt_state625=st)
        params, tiers = game_params(root.config, eng.tiers0)
        o = oracle_c.OracleRealistic(params, tiers, beam_width=width, mt_state625=st, root_w=pack_state(root, eng.tiers0))
        t = 0
        while True:
            a, b = eng.step(), o.step()
            for k in ('n_parents', 'n_raw', 'n_unique', 'n_kept', 'done', 'winner_rank', 'records'):
                assert a[k] == b[k], (goal, t, k, a[k], b[k])
            if a['done']:
                break
            t += 1
            wa, pa, ka = eng.read_turn(t)
            wb, pb, kb = o.turn_arrays(t)
            assert np.array_equal(wa, wb) and np.array_equal(pa, pb) and np.array_equal(ka, kb)
        assert np.array_equal(eng.path_words(), o.path())
        assert np.array_equal(eng.mt_state(), o.mt_state())
        eng.close()
        o.close()
