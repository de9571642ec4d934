"""Drop-in host mirror of the reference's speedrun interface (src/solver.py:203-464).

``State``, ``HEURISTICS`` and ``State.solve`` keep the reference's names, argument
meaning, printing and error behaviour; the beam search itself runs on the MI355X
engine (``engine.BeamEngine`` over ``libsplendor_beam.so``).  Successor
enumeration (``State.__iter__``) also runs on the device.  The Python heuristic
functions are the user-facing per-state scorers (src/solver.py:210-296); inside a
solve the engine evaluates the same formulas on the GPU from host-captured pow
tables, consuming ``random``'s MT19937 stream in the same order as ``sorted``
calls its key, and hands the generator state back to ``random`` afterwards.
"""
from __future__ import annotations

import random
from bisect import insort
from collections.abc import Callable
from random import randint

from . import _lib as L
from . import codec
from .deck import COLOR_NUM, MAX_GEMS, Color, get_deck
from .engine import HEURISTIC_IDS, BeamEngine, device_successors

deck = get_deck()


# ---------------------------------------------------------------- heuristics (src/solver.py:203-305)
def simple_heuristic(state: 'State') -> float:
    """(saved ** 0.4) * (pts ** 2.5) + noise (src/solver.py:210-215)."""
    return (state.saved**0.4) * (state.pts**2.5) + randint(1, 100) * 0.01


def balanced_heuristic(state: 'State') -> float:
    """Points, saved gems, purchasing power, card count, bonus diversity (src/solver.py:218-249)."""
    pts_score = state.pts**2.8
    saved_score = state.saved**0.5
    resources = (sum(state.gems) + sum(state.bonus) * 2) ** 0.3
    card_count = len(state.cards) ** 0.6
    diversity = sum(1 for b in state.bonus if b > 0) ** 0.4
    noise = randint(1, 100) * 0.01
    return pts_score * 100 + saved_score * 10 + resources * 5 + card_count * 3 + diversity * 2 + noise


def aggressive_heuristic(state: 'State') -> float:
    """Heavy weight on points (src/solver.py:252-262)."""
    noise_free = state.pts**3.2 * 200 + state.saved**0.3 * 5 + sum(state.bonus) ** 0.5 * 2
    return noise_free + randint(1, 100) * 0.01


def efficiency_heuristic(state: 'State') -> float:
    """Saved gems and bonuses (src/solver.py:265-286)."""
    pts_score = state.pts**2.0
    saved_score = state.saved**0.7
    bonus_score = sum(state.bonus) ** 1.2
    diversity = sum(1 for b in state.bonus if b > 0) ** 0.8
    noise = randint(1, 100) * 0.01
    return pts_score * 50 + saved_score * 30 + bonus_score * 20 + diversity * 10 + noise


def competitive_heuristic(state: 'State') -> float:
    """Single-player placeholder: the balanced heuristic (src/solver.py:289-296)."""
    return balanced_heuristic(state)


HeuristicFunc = Callable[['State'], float]
HEURISTICS: dict[str, HeuristicFunc] = {
    'simple': simple_heuristic,
    'balanced': balanced_heuristic,
    'aggressive': aggressive_heuristic,
    'efficiency': efficiency_heuristic,
    'competitive': competitive_heuristic,
}
_BUILTIN_IDS = {simple_heuristic: 0, balanced_heuristic: 1, aggressive_heuristic: 2, efficiency_heuristic: 3,
                competitive_heuristic: 1}


def _subtract_with_bonus(gems, cost, bonus):
    """gems - (cost - bonus) and the gems saved (src/gems.py:116-129)."""
    res = []
    saved = 0
    for g, c, b in zip(gems, cost, bonus):
        pay = max(c - b, 0)
        saved += c - pay
        res.append(max(g - pay, 0))
    return tuple(res), saved


# ---------------------------------------------------------------- State (src/solver.py:308-388)
class State:
    """Speedrun state: infinite gem pool, all 90 cards visible."""

    __slots__ = ('cards', 'bonus', 'gems', 'pts', 'saved', 'hash')

    def __init__(self, cards, bonus, gems, pts, saved):
        self.cards = cards
        self.bonus = bonus
        self.gems = gems
        self.pts = pts
        self.saved = saved
        self.hash = hash((self.cards, self.gems))

    @classmethod
    def newgame(cls) -> 'State':
        no_gems = (0,) * COLOR_NUM
        return State(cards=(), bonus=no_gems, gems=no_gems, pts=0, saved=0)

    @classmethod
    def from_packed(cls, lo: int, hi: int) -> 'State':
        cards, bonus, gems, pts, saved = codec.decode(lo, hi)
        return cls(cards, bonus, gems, pts, saved)

    def packed(self) -> tuple[int, int]:
        return codec.encode(self.cards, self.gems, self.pts, self.saved)

    def _packed_checked(self) -> tuple[int, int]:
        """The packed form of a state the engine can expand exactly as the reference would.  The packed
        form derives ``bonus`` from the card set; the reference's ``State(cards, bonus, ...)``
        (src/solver.py:308-318) keeps ``bonus`` as given, and a hand-made one (a head-start bonus, an
        edited field) would expand and score differently: refused, as are card tuples the packed form
        cannot hold (codec.check_cards)."""
        lo, hi = self.packed()
        derived = codec.decode(lo, hi)[1]
        if tuple(self.bonus) != derived:
            raise ValueError(f'State.bonus {tuple(self.bonus)} differs from the bonus implied by State.cards '
                             f'{derived}: the engine derives bonus from the cards and cannot hold a different one')
        return lo, hi

    def __repr__(self):
        if self.cards:
            return f'{self.gems!r} {"-".join(str(deck[c]) for c in self.cards)}'
        return f'{self.gems!r}'

    def __hash__(self):
        return self.hash

    def __eq__(self, other) -> bool:
        return self.hash == other.hash

    def buy_card(self, card_num: int) -> 'State':
        """Buy without an affordability check, as the reference (src/solver.py:338-355)."""
        cards = list(self.cards)
        insort(cards, card_num)
        card = deck[card_num]
        bonus = list(self.bonus)
        bonus[card.bonus.value] += 1
        gems, saved = _subtract_with_bonus(self.gems, card.cost, self.bonus)
        return State(cards=tuple(cards), bonus=tuple(bonus), gems=gems, pts=self.pts + card.pt,
                     saved=self.saved + saved)

    def __iter__(self):
        """Successors in the reference's order — buys in deck order, then takes (src/solver.py:357-388).

        Enumerated on the GPU by the engine's expansion code (``sb_debug_successors``).
        The packed form keeps ``bonus`` implied by ``cards``; states whose ``bonus``
        or ``gems`` were edited by hand are re-packed from their fields.
        """
        lo, hi = self._packed_checked()
        (clo, chi, _), = device_successors([lo], [hi])
        for a, b in zip(clo.tolist(), chi.tolist()):
            yield State.from_packed(a, b)

    # ------------------------------------------------------------ solve (src/solver.py:390-464)
    def solve(self, goal_pts: int = 15, *, use_heuristic: bool = False, heuristic_name: str = 'simple',
              beam_width: int = 300_000, verbose: bool = True, device: int = 0,
              sync_random: bool = True, gpus: int = 1) -> list['State']:
        """Solve the game using BFS with optional heuristic beam search, on the MI355X engine.

        Same signature, output and printing as the reference; ``device`` picks the
        GPU; ``sync_random`` leaves Python's ``random`` where the reference would
        (after one ``randint`` per scored state).  A heuristic registered in
        ``HEURISTICS`` by the user runs as Python on the host over the device's
        next_queue (see ``_host_scores``); the built-in ones run on the device.
        ``gpus > 1`` shards the beam over that many GPUs (devices ``device`` ..
        ``device + gpus - 1``), one worker process each (``multi.launch``); same
        output, same path, same ``random`` state afterwards.
        """
        # everything that can refuse the call is checked before the banner is printed
        heuristic = HEURISTICS.get(heuristic_name, simple_heuristic)
        host_scored = use_heuristic and heuristic not in _BUILTIN_IDS
        if gpus > 1 and host_scored:
            raise ValueError('a user-registered heuristic scores on the host: solve it with gpus=1')
        lo, hi = self._packed_checked()
        if self.hash != hash((self.cards, self.gems)):
            # the reference seeds its trail with this object (src/solver.py:426), i.e. under its stale hash
            raise ValueError('State fields were edited after construction (its hash is stale): the reference '
                             "would seed the trail with the stale hash; build the root with State(...) instead")
        if verbose:
            print('=' * 60)
            print('SPEEDRUN MODE SOLVER')
            print('=' * 60)
            print(f'Target Points: {goal_pts}')
            print(f'Heuristic: {heuristic_name if use_heuristic else "None (pure BFS)"}')
            if use_heuristic:
                print(f'Beam Width: {beam_width:,}')
            print('Gem Pool: Infinite')
            print('Card Visibility: All 90 cards')
            print('=' * 60)
            print()
        hid = _BUILTIN_IDS.get(heuristic, 0) if use_heuristic else 0
        if host_scored:
            # a user-registered callable (HEURISTICS.md:204-229): the device expands and dedups; the callable
            # scores next_queue on the host, in next_queue order (the order `sorted` calls its key in, so it
            # consumes `random` exactly as the reference); the device runs the stable top-k of its scores
            hid = L.SB_HEUR_HOST
        st = random.getstate()
        if gpus > 1:
            from .multi import launch
            res = launch({'goal': goal_pts, 'use_heuristic': bool(use_heuristic), 'heuristic': hid,
                          'beam_width': beam_width, 'mt': list(st[1]), 'root': [lo, hi], 'verbose': verbose,
                          'device': device}, gpus)
            if use_heuristic and sync_random:
                random.setstate((st[0], tuple(int(x) for x in res['mt']), st[2]))
            return [State.from_packed(a, b) for a, b in res['path']]
        eng = BeamEngine(goal_pts=goal_pts, use_heuristic=use_heuristic, heuristic=hid, beam_width=beam_width,
                         mt_state625=st[1], root_lo=lo, root_hi=hi, device=device)
        try:
            turn = 0
            while True:
                if verbose:
                    print(f'turn={turn:<10} {State.from_packed(*eng.state_at(turn, 0))}')
                stats = eng.step()
                if verbose:
                    for rank, pts in stats['records']:
                        print(f'max_pts={pts:<7} {State.from_packed(*eng.state_at(turn, rank))}')
                if stats['done']:
                    break
                if eng.host_scored:
                    eng.prune(_host_scores(eng, heuristic))
                turn += 1
            path = [State.from_packed(a, b) for a, b in eng.path()]
            if use_heuristic and sync_random and not eng.host_scored:
                mt = eng.mt_state()
                random.setstate((st[0], tuple(int(x) for x in mt), st[2]))
        finally:
            eng.close()
        return path


def _host_scores(eng: BeamEngine, heuristic, chunk: int = 1 << 20):
    """The callable's score of every next_queue entry, in next_queue order, as float64.  Python compares the
    returned values exactly; a value float64 cannot hold exactly (an int beyond 2**53) would be ordered
    differently on the device, so it is refused."""
    import numpy as np
    out = np.empty(eng.pending, dtype=np.float64)
    for a in range(0, eng.pending, chunk):
        lo, hi = eng.read_next(a, min(chunk, eng.pending - a))
        for i, (x, y) in enumerate(zip(lo.tolist(), hi.tolist())):
            v = heuristic(State.from_packed(x, y))
            f = float(v)
            if type(v) is not float and f != v:
                raise TypeError(f'heuristic returned {v!r}, which float64 cannot represent exactly')
            out[a + i] = f
    return out


__all__ = ['State', 'HEURISTICS', 'simple_heuristic', 'balanced_heuristic', 'aggressive_heuristic',
           'efficiency_heuristic', 'competitive_heuristic', 'Color', 'MAX_GEMS']
