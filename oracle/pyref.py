"""Pure-Python, single-threaded restatement of the reference's speedrun beam step — TEST INFRASTRUCTURE.

This is the CPU path the way the reference runs it: CPython objects, the interpreter's own tuple hash
for the trail, `random.randint` noise and a stable `sorted`, one core.  `bench.py`'s `cpu_baseline` leg
times it beside the C oracle (the reference itself cannot travel to the GPU box); `tests/test_pyref.py`
pins it to the reference's captures (successor lists, seeded solves: beam digests, paths, MT state).
The product path (`splendor-rl-gym_amd/`) never imports it.

Restated from IamJasonBian/Splendor-RL-Gym:
  identity   hash((cards, gems)), cards a sorted tuple            src/solver.py:318,332-336
  successors buys in deck order (cost <= min(g+b, 7), not owned),  src/solver.py:357-388,
             then takes from the bucketed pattern table              src/buys.py:13-17, src/gems.py:14-113
  buy        c = max(cost-bonus, 0); saved += cost-c; gems -= c      src/solver.py:338-355, src/gems.py:116-143
  heuristics simple / balanced / aggressive / efficiency           src/solver.py:210-305
  turn loop  goal check, trail dedup, stable prune to W            src/solver.py:425-464
"""
from __future__ import annotations

import hashlib
import os
import random
import sys
from itertools import permutations

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(os.path.dirname(HERE), 'splendor-rl-gym_amd')
if PKG_ROOT not in sys.path:
    sys.path.insert(0, PKG_ROOT)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))   # ref_tables beside this file
from ref_tables import deck_rows  # noqa: E402  (the captured deck, not the product's deck.py)

MAXG = 7
_ROWS = list(deck_rows())   # 7 ints per card: cost[5], pt, colour
DECK = [(tuple(_ROWS[7 * c:7 * c + 5]), _ROWS[7 * c + 5], _ROWS[7 * c + 6]) for c in range(90)]   # deck order

# take patterns per gem-total bucket in the reference's order (src/gems.py:22-37, 85-108):
# take-3 family first, then take-2; each family in distinct-permutation (lexicographic) order
_FAMILIES = {
    7: [(1, 1, 1, 0, 0)], 8: [(1, 1, 1, -1, 0), (1, 1, 0, 0, 0)],
    9: [(1, 1, 1, -1, -1), (1, 1, -1, 0, 0), (1, 0, 0, 0, 0)], 10: [(1, 1, -1, -1, 0), (1, -1, 0, 0, 0)]}
_TWOS = {7: [(2, 0, 0, 0, 0)], 8: [(2, 0, 0, 0, 0)], 9: [(2, -1, 0, 0, 0)], 10: [(2, -1, -1, 0, 0), (2, -2, 0, 0, 0)]}


def _perms(p):
    return sorted(set(permutations(p)))


PATTERNS = {b: [(d, None) for f in _FAMILIES[b] for d in _perms(f)] +
               [(d, d.index(2)) for f in _TWOS[b] for d in _perms(f)] for b in _FAMILIES}

_takes_cache: dict = {}
_buys_cache: dict = {}


def takes(gems):
    """Successor gem tuples of `gems` (get_takes()[gems]): valid iff every colour stays in 0..7 and a
    take-2 colour held at most 3 before."""
    t = _takes_cache.get(gems)
    if t is None:
        s = sum(gems)
        t = []
        if s <= 10:
            for d, two in PATTERNS[min(max(s, 7), 10)]:
                if two is not None and gems[two] > MAXG - 4:
                    continue
                ng = tuple(g + x for g, x in zip(gems, d))
                if all(0 <= x <= MAXG for x in ng):
                    t.append(ng)
        _takes_cache[gems] = t
    return t


def buys(cap):
    """Cards affordable with the capped purchasing power `cap` = min(gems + bonus, 7), deck order."""
    b = _buys_cache.get(cap)
    if b is None:
        b = [c for c, (cost, _, _) in enumerate(DECK) if all(x <= y for x, y in zip(cost, cap))]
        _buys_cache[cap] = b
    return b


class PState:
    """Speedrun state: cards (sorted tuple), bonus, gems, pts, saved (src/solver.py:308-336)."""
    __slots__ = ('cards', 'bonus', 'gems', 'pts', 'saved', 'key')

    def __init__(self, cards, bonus, gems, pts, saved):
        self.cards, self.bonus, self.gems, self.pts, self.saved = cards, bonus, gems, pts, saved
        self.key = hash((cards, gems))

    def children(self):
        cards, bonus, gems = self.cards, self.bonus, self.gems
        cap = tuple(min(g + b, MAXG) for g, b in zip(gems, bonus))
        for c in buys(cap):
            if c in cards:
                continue
            cost, pt, colour = DECK[c]
            paid = [max(x - b, 0) for x, b in zip(cost, bonus)]
            saved = self.saved + sum(x - p for x, p in zip(cost, paid))
            nb = list(bonus)
            nb[colour] += 1
            yield PState(tuple(sorted(cards + (c,))), tuple(nb), tuple(max(g - p, 0) for g, p in zip(gems, paid)),
                         self.pts + pt, saved)
        for ng in takes(gems):
            yield PState(cards, bonus, ng, self.pts, self.saved)


def _noise(rng):
    return rng.randint(1, 100) * 0.01


def h_simple(s, rng):
    return s.saved ** 0.4 * s.pts ** 2.5 + _noise(rng)


def h_balanced(s, rng):
    B = sum(s.bonus)
    U = sum(1 for b in s.bonus if b > 0)
    return (s.pts ** 2.8 * 100 + s.saved ** 0.5 * 10 + (sum(s.gems) + B * 2) ** 0.3 * 5 + len(s.cards) ** 0.6 * 3
            + U ** 0.4 * 2 + _noise(rng))


def h_aggressive(s, rng):
    return s.pts ** 3.2 * 200 + s.saved ** 0.3 * 5 + sum(s.bonus) ** 0.5 * 2 + _noise(rng)


def h_efficiency(s, rng):
    U = sum(1 for b in s.bonus if b > 0)
    return s.pts ** 2.0 * 50 + s.saved ** 0.7 * 30 + sum(s.bonus) ** 1.2 * 20 + U ** 0.8 * 10 + _noise(rng)


HEURISTICS = {'simple': h_simple, 'balanced': h_balanced, 'aggressive': h_aggressive, 'efficiency': h_efficiency,
              'competitive': h_balanced}


class PySolve:
    """Stepwise beam solve (src/solver.py:390-464) with the same step record as the C oracle."""

    def __init__(self, goal_pts, *, use_heuristic, heuristic_name, beam_width, mt_state625=None, rng=None,
                 root=None):
        self.goal, self.use_heuristic, self.width = goal_pts, use_heuristic, beam_width
        self.heur = HEURISTICS.get(heuristic_name, h_simple)   # unknown name -> simple (:429)
        if rng is None:
            rng = random.Random()
            rng.setstate((3, tuple(int(x) for x in mt_state625), None))
        self.rng = rng
        root = root or PState((), (0,) * 5, (0,) * 5, 0, 0)
        self.trail = {root.key}
        self.turns = [([root], [None])]
        self.done, self.winner_rank = False, -1

    def step(self) -> dict:
        queue, _ = self.turns[-1]
        out = {'n_parents': len(queue), 'n_raw': 0, 'n_unique': 0, 'n_kept': 0, 'done': False, 'winner_rank': -1}
        for r, s in enumerate(queue):               # goal check in queue order (:438-445)
            if s.pts >= self.goal:
                self.done, self.winner_rank = True, r
                out.update(done=True, winner_rank=r)
                return out
        trail, nxt, par, raw = self.trail, [], [], 0
        for r, s in enumerate(queue):               # expansion + trail dedup (:446-450)
            for ch in s.children():
                raw += 1
                if ch.key in trail:
                    continue
                trail.add(ch.key)
                nxt.append(ch)
                par.append(r)
        out.update(n_raw=raw, n_unique=len(nxt))
        if not nxt:                                  # queue empties: the last parent ends the search
            self.done, self.winner_rank = True, len(queue) - 1
            out.update(done=True, winner_rank=len(queue) - 1)
            return out
        if self.use_heuristic:                       # sorted(next_queue, key=heuristic, reverse=True)[:W]
            h, rng = self.heur, self.rng
            score = [h(s, rng) for s in nxt]
            order = sorted(range(len(nxt)), key=score.__getitem__, reverse=True)[:self.width]
            nxt, par = [nxt[i] for i in order], [par[i] for i in order]
        self.turns.append((nxt, par))
        out['n_kept'] = len(nxt)
        return out

    def keys(self, t) -> np.ndarray:
        return np.array([s.key for s in self.turns[t][0]], dtype=np.int64).view(np.uint64)

    def path(self):
        t, r, out = len(self.turns) - 1, self.winner_rank, []
        while t >= 0:
            queue, par = self.turns[t]
            out.append(queue[r])
            r = par[r]
            t -= 1
        return out[::-1]

    def mt_state(self):
        st = self.rng.getstate()[1]
        return np.array(st, dtype=np.uint32)


def beam_digest(keys_u64: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(keys_u64, dtype=np.uint64).view('<i8').tobytes()).hexdigest()[:16]


def state_from_packed(lo: int, hi: int) -> PState:
    """PState from the engine's packed (lo, hi) words (include/splendor_beam.h layout)."""
    cards = []
    m = lo
    while m:
        b = m & -m
        cards.append(b.bit_length() - 1)
        m ^= b
    m = hi & ((1 << 26) - 1)
    while m:
        b = m & -m
        cards.append(63 + b.bit_length())
        m ^= b
    bonus = [0] * 5
    for c in cards:
        bonus[DECK[c][2]] += 1
    gems = tuple((hi >> (26 + 3 * i)) & 7 for i in range(5))
    return PState(tuple(cards), tuple(bonus), gems, (hi >> 41) & 0xFF, hi >> 49)


def from_oracle(o, goal_pts, heuristic_name, beam_width, sample=None) -> PySolve:
    """A PySolve continuing the C oracle `o` from its newest beam: same queue, same trail, same MT state
    (bench.py times one saturated step of it without replaying the early turns in Python).  sample = k: only
    the beam's first k parents, and a trail of the newest beam's keys instead of every visited key (a bounded
    timing sample of a wide turn: the Python trail of a W=4M solve would not fit; a child found in an older turn
    is then scored and sorted as new, so the sample's rate errs low)."""
    t = o.nturns() - 1
    lo, hi, _, key = o.turn_arrays(t)
    if sample is not None:
        lo, hi = lo[:sample], hi[:sample]
    beam = [state_from_packed(a, b) for a, b in zip(lo.tolist(), hi.tolist())]
    ps = PySolve(goal_pts, use_heuristic=True, heuristic_name=heuristic_name, beam_width=beam_width,
                 mt_state625=o.mt_state())
    ps.trail = set((key if sample is not None else o.visited_keys()).view(np.int64).tolist())
    ps.turns = [(beam, [None] * len(beam))]
    return ps
