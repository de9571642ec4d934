"""The oracle's own tables and state packing (TEST INFRASTRUCTURE).

The checker must not share the product's tables: the deck comes from the fixture captured by importing the
reference itself (tests/golden/tables.json 'deck': cost, pt, colour per card in the reference's deck order,
src/cardparser.py:17-66 over cards.csv:2-91, written by tests/golden/make_golden.py), and the packed (lo, hi) state
the oracle exchanges with the tests is restated here — cards 0..63 in lo, cards 64..89 in hi bits 0-25, gem i in bits
26+3i, pts in 41-48, saved in 49-63 — not imported from splendor_amd.codec.  Only tests/, smoke()
and bench.py's cpu_baseline use it.
"""
from __future__ import annotations

import json
import os
from functools import lru_cache

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLES = os.path.join(REPO, 'tests', 'golden', 'tables.json')
NCOL = 5


@lru_cache(maxsize=None)
def deck():
    """[(cost tuple, pt, colour)] per card, in the reference's deck order (the captured fixture)."""
    with open(TABLES) as f:
        d = json.load(f)['deck']
    assert len(d) == 90, 'the captured deck holds 90 cards'
    return tuple((tuple(int(x) for x in c['cost']), int(c['pt']), int(c['color'])) for c in d)


def deck_rows() -> list[int]:
    """Flat cost[5], pt, colour per card (the layout oc_init and the pure-Python restatement read)."""
    out: list[int] = []
    for cost, pt, col in deck():
        out.extend(cost)
        out.append(pt)
        out.append(col)
    return out


def to_signed(k: int) -> int:
    return k - (1 << 64) if k >= (1 << 63) else k


def encode(cards, gems, pts: int, saved: int) -> tuple[int, int]:
    lo = hi = 0
    prev = -1
    for c in cards:
        c = int(c)
        assert 0 <= c < 90 and c > prev, f'cards {tuple(cards)}: ids in 0..89, ascending, distinct'
        prev = c
        if c < 64:
            lo |= 1 << c
        else:
            hi |= 1 << (c - 64)
    assert len(gems) == NCOL and all(0 <= g <= 7 for g in gems), gems
    for i, g in enumerate(gems):
        hi |= int(g) << (26 + 3 * i)
    assert 0 <= pts < 256 and 0 <= saved < (1 << 15), (pts, saved)
    return lo, hi | (int(pts) << 41) | (int(saved) << 49)


def decode(lo: int, hi: int):
    """-> (cards tuple sorted, bonus, gems, pts, saved)."""
    cards = tuple([c for c in range(64) if lo >> c & 1] + [64 + c for c in range(26) if hi >> c & 1])
    gems = tuple((hi >> (26 + 3 * i)) & 7 for i in range(NCOL))
    bonus = [0] * NCOL
    dk = deck()
    for c in cards:
        bonus[dk[c][2]] += 1
    return cards, tuple(bonus), gems, (hi >> 41) & 0xFF, hi >> 49
