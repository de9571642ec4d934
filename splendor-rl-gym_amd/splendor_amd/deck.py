"""The 90-card Splendor deck and colour constants (game data).

Mirrors the reference's data layer: ``Color`` (src/color.py:4-15), ``Card`` /
``get_deck`` (src/cardparser.py:17-66) and ``cards.csv``.  The deck is encoded
here as one token per card, in deck-index order: five cost digits (white, blue,
green, red, black), the point value, and the bonus colour letter
(W=white, U=blue, G=green, R=red, K=black).  ``tests/test_tables.py`` pins it
against the golden capture (``tests/golden/tables.json``).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from functools import cache

COLOR_NUM = 5
MAX_GEMS = 7


class Color(enum.Enum):
    """Gem colours, value = index into every 5-vector (src/color.py:4-12)."""

    WHITE = 0
    BLUE = 1
    GREEN = 2
    RED = 3
    BLACK = 4

    def __repr__(self):
        return self.__str__()


_DECK_TOKENS = """
    030000W 000030U 000300G 300000R 003000K 000210W 100020U 210000G 021000R 002100K
    020020W 002020U 020200G 200200R 202000K 011110W 101110U 110110G 111010R 111100K
    310010W 013100U 131000G 100130R 001310K 022010W 102200U 010220G 201020R 220100K
    012110W 101210U 110120G 211010R 121100K 004001W 000401U 000041G 400001R 040001K
    003221W 022301U 230021G 200231R 322001K 230301W 023031U 302301G 030231R 303021K
    000502W 050002U 005002G 000052R 500002K 001422W 200142U 420012G 142002R 014202K
    000532W 530002U 053002G 300052R 005302K 600003W 060003U 006003G 000603R 000063K
    033533W 303353U 530333G 353033R 335303K 000074W 700004U 070004G 007004R 000704K
    300364W 630034U 363004G 036304R 003634K 300075W 730005U 073005G 007305R 000735K
"""
_LETTER = {'W': Color.WHITE, 'U': Color.BLUE, 'G': Color.GREEN, 'R': Color.RED, 'K': Color.BLACK}


@dataclass(frozen=True)
class Card:
    """One development card (src/cardparser.py:17-46)."""

    cost: tuple[int, ...]
    pt: int
    bonus: Color
    index: int

    @property
    def str_id(self) -> str:
        """Points, colour letter (K for black), sorted non-zero costs — e.g. ``1W223``."""
        letter = 'K' if self.bonus is Color.BLACK else self.bonus.name[0]
        return f'{self.pt}{letter}' + ''.join(sorted(str(x) for x in self.cost if x))

    def __str__(self):
        return self.str_id

    def __hash__(self):
        return self.index

    def __eq__(self, other):
        return self.index == other.index


@cache
def get_deck() -> tuple[Card, ...]:
    toks = _DECK_TOKENS.split()
    assert len(toks) == 90
    return tuple(Card(cost=tuple(int(ch) for ch in t[:5]), pt=int(t[5]), bonus=_LETTER[t[6]], index=i)
                 for i, t in enumerate(toks))


def deck_rows() -> list[int]:
    """Flat int rows ``cost[5], pt, colour`` per card — the layout of ``sb_init_tables``."""
    out: list[int] = []
    for c in get_deck():
        out.extend(c.cost)
        out.append(c.pt)
        out.append(c.bonus.value)
    return out
