"""GPU parity tests: the HIP engine (through the C-ABI) against the CPU oracle and the reference's goldens.

Bit-exact bar: successor lists, keys, scores (float64 bits), MT words, per-turn beams
(keys + parent links), solution paths and the final MT19937 state.
"""
import random

import numpy as np
import pytest

import oracle_c
from conftest import golden, golden_exists
from splendor_amd import codec
from splendor_amd.engine import BeamEngine, device_mt_words, device_scores, device_successors, device_topk

pytestmark = pytest.mark.gpu


def _mt(seed):
    random.seed(seed)
    return random.getstate()[1]


# ---------------------------------------------------------------- kernels
def test_device_successors_golden(tables):
    """k_expand enumeration == reference State.__iter__ (order, states, hash) on the captured parents."""
    par = [s['parent'] for s in tables['successors']]
    lo, hi = zip(*[codec.encode(p[0], p[2], p[3], p[4]) for p in par])
    out = device_successors(lo, hi)
    for s, (clo, chi, ckey) in zip(tables['successors'], out):
        got = [(*codec.decode(int(a), int(b)), codec.to_signed(int(k))) for a, b, k in zip(clo, chi, ckey)]
        exp = [(tuple(c[0]), tuple(c[1]), tuple(c[2]), c[3], c[4], c[5]) for c in s['children']]
        assert got == exp


def test_device_successors_random_vs_oracle():
    """Random reachable-ish states (all gem totals 0..10, 0..25 cards)."""
    rng = np.random.default_rng(1)
    lo, hi = [], []
    for _ in range(3000):
        cards = sorted(rng.choice(90, rng.integers(0, 26), replace=False).tolist())
        while True:
            gems = rng.integers(0, 8, 5).tolist()
            if sum(gems) <= 10:
                break
        a, b = codec.encode(cards, gems, int(rng.integers(0, 40)), int(rng.integers(0, 200)))
        lo.append(a)
        hi.append(b)
    out = device_successors(lo, hi)
    L = oracle_c.lib()
    olo = np.zeros(256, np.uint64)
    ohi = np.zeros(256, np.uint64)
    okey = np.zeros(256, np.uint64)
    for i, (clo, chi, ckey) in enumerate(out):
        n = L.oc_successors(lo[i], hi[i], olo, ohi, okey)
        assert n == len(clo)
        assert np.array_equal(clo, olo[:n]) and np.array_equal(chi, ohi[:n]) and np.array_equal(ckey, okey[:n])


def test_device_mt_words(tables):
    for seed, v in tables['mt'].items():
        st = np.array(v['state'], np.uint32)
        w = device_mt_words(st, 2000)
        assert w.tolist() == v['words']
    # a long run crossing many device twists vs the oracle's host MT
    random.seed(777)
    for _ in range(313):
        random.getrandbits(32)
    st = random.getstate()[1]
    w = device_mt_words(st, 200_000)
    ref = np.zeros(200_000, np.uint32)
    oracle_c.lib().oc_mt_words(np.array(st, np.uint32), ref, 200_000)
    assert np.array_equal(w, ref)


@pytest.mark.parametrize('producers,twists,n', [(1, 1, 5000), (4, 3, 50_000), (8, 1, 31_000), (256, 2, 400_000),
                                                (256, 64, 25_000_000)])
def test_device_mt_jump_ahead(producers, twists, n):
    """Jump-ahead producers (doubling tree + chunk stride) reproduce the sequential stream word for word."""
    random.seed(producers * 1000 + twists)
    for _ in range(17):
        random.getrandbits(32)
    st = random.getstate()[1]
    w = device_mt_words(st, n, producers=producers, twists=twists)
    ref = np.zeros(n, np.uint32)
    oracle_c.lib().oc_mt_words(np.array(st, np.uint32), ref, n)
    assert np.array_equal(w, ref)


@pytest.mark.parametrize('hid,name', [(0, 'simple'), (1, 'balanced'), (2, 'aggressive'), (3, 'efficiency'),
                                      (1, 'competitive')])
def test_device_scores_golden(tables, hid, name):
    rows = tables['heuristic_scores_seed11']
    random.seed(11)
    k = random.randint(1, 100)
    lo, hi = zip(*[codec.encode(r['cards'], r['gems'], r['pts'], r['saved']) for r in rows])
    got = device_scores(hid, lo, hi, [k] * len(rows))
    assert [float(x).hex() for x in got] == [r[name] for r in rows]


def test_device_topk_stable():
    rng = np.random.default_rng(5)
    for n, keep, distinct in [(1, 1, 1), (1000, 10, 3), (50_000, 7_000, 40), (300_000, 300_000, 1000),
                              (1_000_000, 123_457, 2500), (200_000, 1, 5), (70_000, 69_999, 2),
                              (3_000_000, 2_600_000, 200_000)]:   # >= 256 sort tiles: the two-level passes
        vals = rng.choice(rng.random(distinct) * 1e4 + 0.01, n)
        keys = vals.astype(np.float64).view(np.uint64)
        exp = np.argsort(-vals, kind='stable')[:keep]
        got = device_topk(keys, keep)
        assert np.array_equal(got, exp.astype(np.uint32)), (n, keep, distinct)


def test_device_oe_merge_segments():
    """The owner-emission receive merge (sb_oe.inc k_oe_merge) against a sort of the positions: segments of
    ascending, distinct positions, evenly interleaved, a sparse segment beside dense ones (the per-lane
    fallback past OE_MERGE_SPAN), empty segments, a single segment, 64 segments, runs of 64 and off-by-one sizes."""
    import ctypes as C
    from splendor_amd import _lib
    rng = np.random.default_rng(11)

    def case(sizes, spread):
        m = int(sum(sizes))
        pos = rng.choice(spread, m, replace=False).astype(np.uint32)
        owner = rng.permutation(np.repeat(np.arange(len(sizes)), sizes))   # which segment each position joins
        segs = [np.sort(pos[owner == q]) for q in range(len(sizes))]
        flat = np.ascontiguousarray(np.concatenate(segs).astype(np.uint32))
        start = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        out = np.empty(m, np.uint32)
        _lib.check(_lib.lib().sb_debug_oe_merge(0, flat, m, len(sizes), start, out), 'sb_debug_oe_merge')
        assert np.array_equal(out, np.argsort(flat, kind='stable').astype(np.uint32)), sizes[:8]

    case([100_000], 10**6)
    case([50_000] * 8, 2**31)
    case([1, 2, 63, 64, 65, 127, 128, 129], 10**4)
    case([300_000, 17, 300_000, 0, 5, 200_000, 3, 0], 2**32 - 1)   # sparse segments among dense ones
    case([0, 0, 4096, 0], 10**5)
    case(list(rng.integers(0, 3000, 64)), 10**7)


def test_device_topk_key_ranges():
    """Select/sort over u64 keys spanning the full range, all-equal keys, keys differing only in low
    bits, keep > n, and a threshold inside a heavily tied bucket (stable descending order)."""
    rng = np.random.default_rng(9)
    cases = [
        rng.integers(0, 2**64 - 1, 300_000, dtype=np.uint64, endpoint=True),                 # full range
        np.full(50_000, 12345, dtype=np.uint64),                                               # all equal
        (np.uint64(0x4010_0000_0000_0000) + rng.integers(0, 4, 200_000).astype(np.uint64)),  # low bits
        np.repeat(rng.integers(0, 2**63, 7).astype(np.uint64), 30_000),                         # 7 values
        rng.choice(np.array([0, 1, 2**63, 2**64 - 1], dtype=np.uint64), 100_000),              # extremes
    ]
    for keys in cases:
        n = len(keys)
        for keep in (1, n // 3, n - 1, n, n + 5):
            exp = np.lexsort((np.arange(n), ~keys))[:min(keep, n)]
            got = device_topk(keys, keep)
            assert np.array_equal(got, exp.astype(np.uint32)), (n, keep, keys[:3])


def test_device_topk_prefix_fixup():
    """The sort orders 32-bit prefixes of the varying bits, then fixes runs of equal prefixes that hold
    different keys: keys spanning > 32 bits where many differ only below the prefix, with heavy ties,
    a hot value sharing its prefix with others, runs longer than a workgroup, and runs at both ends."""
    rng = np.random.default_rng(21)
    base = np.uint64(0x40E0_0000_0000_0000)
    cases = []
    hi = rng.integers(0, 2**12, 400_000).astype(np.uint64) << np.uint64(40)    # 52 varying bits
    lo = rng.integers(0, 3, 400_000).astype(np.uint64) * np.uint64(7)          # below the 32-bit prefix
    cases.append(base + hi + lo)
    hot = np.concatenate([np.full(20_000, 5, np.uint64), np.full(3_000, 6, np.uint64), np.full(9_000, 4, np.uint64),
                          rng.integers(0, 2**50, 30_000).astype(np.uint64)])
    cases.append(base + hot[rng.permutation(len(hot))])                         # long mixed run + spread keys
    few = rng.integers(0, 2**44, 64).astype(np.uint64)
    cases.append(base + rng.choice(few, 250_000) + rng.integers(0, 2, 250_000).astype(np.uint64))
    for keys in cases:
        n = len(keys)
        for keep in (n // 5, n, n + 1):
            exp = np.lexsort((np.arange(n), ~keys))[:min(keep, n)]
            got = device_topk(keys, keep)
            assert np.array_equal(got, exp.astype(np.uint32)), (n, keep)


# ---------------------------------------------------------------- whole solves
def _run_pair(goal, heur, width, seed, use_heuristic=True, test_flags=0):
    from splendor_amd.engine import HEURISTIC_IDS
    st = _mt(seed)
    eng = BeamEngine(goal_pts=goal, use_heuristic=use_heuristic, heuristic=HEURISTIC_IDS.get(heur, 0),
                     beam_width=width, mt_state625=st, test_flags=test_flags)
    return eng, st


def _skey(lo, hi):
    cards, _, gems, _, _ = codec.decode(lo, hi)
    return codec.to_signed(codec.state_key(cards, gems))


def _check_against_golden(g, test_flags=0):
    eng, _ = _run_pair(g['goal'], g['heuristic'], g['beam_width'], g['seed'], test_flags=test_flags)
    turns = [t for t in g['turns'] if t['n_unique'] > 0]
    t = 0
    while True:
        stt = eng.step()
        if stt['done']:
            break
        t += 1
        exp = turns[t - 1]
        assert stt['n_unique'] == exp['n_unique'], t
        _, _, _, key = eng.read_turn(t)
        assert len(key) == exp['n_kept'] and oracle_c.beam_digest(key) == exp['digest'], f'turn {t}'
    assert t == len(turns)
    path = eng.path()
    assert [_skey(a, b) for a, b in path] == [p[5] for p in g['path']]
    assert oracle_c.mt_fingerprint(eng.mt_state()) == g['final_mt']
    eng.close()


def test_solves_small_golden():
    for g in golden('solves_small.json'):
        _check_against_golden(g)


@pytest.mark.parametrize('name', ['solve_g10_simple_w300000_s0.json', 'solve_g15_simple_w300000_s0.json',
                                  'solve_g15_balanced_w300000_s0.json', 'solve_g15_aggressive_w300000_s0.json',
                                  'solve_g15_efficiency_w300000_s0.json'])
def test_solve_w300k_golden(name):
    if not golden_exists(name):
        pytest.skip(f'{name} not captured')
    _check_against_golden(golden(name))


@pytest.mark.parametrize('flags', [4, 8])
def test_solve_select_paths_golden(flags):
    """The top-k's first select pass three ways: folded into the emission (every other solve test), the
    generic pass (flags bit 2), and the folded pass with its window forced off the keys so that its
    fallback runs (bit 3) — same beams every turn."""
    _check_against_golden(golden('solve_g15_efficiency_w300000_s0.json'), test_flags=flags)
    for g in golden('solves_small.json')[:6]:
        _check_against_golden(g, test_flags=flags)


def test_solve_c3_w4m_oracle_golden():
    """Config C3 (goal 15 -u -H balanced W=4M seed 0): the reference cannot run it here (RAM), so the
    golden is the C oracle's (itself pinned to the reference's W<=300k captures)."""
    g = golden('oracle_g15_balanced_w4000000_s0.json')
    assert g['moves'] == 15
    _check_against_golden(g)


def test_solve_efficiency_w4m_oracle_golden():
    """C5's heuristic (efficiency) at C3's width on one GPU: the golden the sharded W=4M test also uses."""
    g = golden('oracle_g15_efficiency_w4000000_s0.json')
    assert g['moves'] == 15
    _check_against_golden(g)


def test_bfs_golden():
    for g in golden('bfs.json'):
        eng = BeamEngine(goal_pts=g['goal'], use_heuristic=False, heuristic=0, beam_width=1, mt_state625=_mt(0))
        while not eng.step()['done']:
            pass
        path = [repr_state(a, b) for a, b in eng.path()]
        assert path == [p[4] for p in g['path']]
        eng.close()


def repr_state(lo, hi):
    from splendor_amd.solver import State
    return repr(State.from_packed(lo, hi))


def test_vs_oracle_stepwise_random_configs():
    """Per-turn beams (keys AND parent links) identical to the C oracle over several configs."""
    for goal, heur, width, seed in [(8, 'simple', 5000, 3), (9, 'efficiency', 20000, 4), (7, 'aggressive', 777, 5),
                                    (12, 'balanced', 50000, 6)]:
        eng, st = _run_pair(goal, heur, width, seed)
        ora = oracle_c.OracleSolve(goal, use_heuristic=True, heuristic_name=heur, beam_width=width, mt_state625=st)
        t = 0
        while True:
            a, b = eng.step(), ora.step()
            for k in ('n_parents', 'n_raw', 'n_unique', 'n_kept', 'done', 'winner_rank', 'records'):
                assert a[k] == b[k], (goal, heur, t, k)
            if a['done']:
                break
            t += 1
            _, _, pa, ka = eng.read_turn(t)
            _, _, pb, kb = ora.turn_arrays(t)
            assert np.array_equal(ka, kb) and np.array_equal(pa, pb)
        assert eng.path() == ora.path()
        assert np.array_equal(eng.mt_state(), ora.mt_state())
        eng.close()
        ora.close()


def test_saved_overflow_is_an_error_not_a_clamp():
    """saved >= 256 is past the pow tables: the step fails loudly instead of scoring with a clamped value."""
    from splendor_amd import _lib as L
    from splendor_amd.codec import encode
    lo, hi = encode((), (0, 0, 0, 0, 0), 0, 300)
    eng = BeamEngine(goal_pts=15, use_heuristic=True, heuristic=1, beam_width=100, mt_state625=_mt(0),
                     root_lo=lo, root_hi=hi)
    eng.step()   # turn 0: the root's children are scored in this step's emission
    with pytest.raises(L.SplendorBeamError, match='saved >= 256'):
        for _ in range(3):
            eng.step()
    eng.close()


def test_solve_lookahead_toggled_golden():
    """sb_set_lookahead (the bench switches it at the edges of its timed window): with the next turn's
    expansion launched at the end of a step or at the start of the next, in any pattern, the beams,
    path and MT state stay the golden's."""
    rng = np.random.default_rng(7)
    for g in [golden('solve_g15_balanced_w300000_s0.json')] + golden('solves_small.json')[:4]:
        eng, _ = _run_pair(g['goal'], g['heuristic'], g['beam_width'], g['seed'])
        turns = [t for t in g['turns'] if t['n_unique'] > 0]
        t = 0
        while True:
            eng.set_lookahead(bool(rng.integers(2)))
            stt = eng.step()
            if stt['done']:
                break
            t += 1
            _, _, _, key = eng.read_turn(t)
            assert oracle_c.beam_digest(key) == turns[t - 1]['digest'], f'turn {t}'
        assert t == len(turns)
        assert [_skey(a, b) for a, b in eng.path()] == [p[5] for p in g['path']]
        assert oracle_c.mt_fingerprint(eng.mt_state()) == g['final_mt']
        eng.close()
