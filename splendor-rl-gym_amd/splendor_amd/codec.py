"""Packed speedrun-state codec shared by the host, the HIP engine and the oracle.

A speedrun ``State`` (src/solver.py:308-318: cards, bonus, gems, pts, saved) is
stored on the device as two little-endian u64 words (``include/splendor_beam.h``):

* ``lo``  — owned-card bitmask, cards 0..63
* ``hi``  — bits 0..25 cards 64..89 | bits 26+3i gem count of colour i (0..7)
           | bits 41..48 pts | bits 49..63 saved

``bonus`` is derived from the card mask (one card = +1 bonus of its colour), as
in the reference where ``bonus`` only changes in ``buy_card`` (src/solver.py:346).
The identity key is CPython's 64-bit ``hash((cards, gems))`` (src/solver.py:318),
restated exactly in :func:`state_key`.
"""
from __future__ import annotations

from .deck import COLOR_NUM, get_deck

_M64 = (1 << 64) - 1
XXP1 = 11400714785074694791
XXP2 = 14029467366897019727
XXP5 = 2870177450012600261


def _tuplehash(lanes) -> int:
    """CPython ``tuplehash`` (Objects/tupleobject.c, 3.8+) on unsigned 64-bit lanes."""
    acc = XXP5
    n = 0
    for lane in lanes:
        acc = (acc + (lane & _M64) * XXP2) & _M64
        acc = ((acc << 31) | (acc >> 33)) & _M64
        acc = (acc * XXP1) & _M64
        n += 1
    acc = (acc + (n ^ (XXP5 ^ 3527539))) & _M64
    return 1546275796 if acc == _M64 else acc


def state_key(cards, gems) -> int:
    """Unsigned 64-bit ``hash((cards, gems))``; ``to_signed`` gives Python's ``hash`` value."""
    return _tuplehash((_tuplehash(cards), _tuplehash(gems)))


def to_signed(k: int) -> int:
    return k - (1 << 64) if k >= (1 << 63) else k


def check_cards(cards) -> None:
    """The packed form holds a card SET; refuse a ``cards`` tuple it would silently change.

    The reference keeps ``cards`` as a tuple built by ``insort`` (src/solver.py:343), hashes that tuple
    (:318) and never checks ownership in ``buy_card`` (:338-355).  A tuple with an id outside 0..89, a
    repeated id or ids out of order would be re-ordered / collapsed / mis-packed here, giving a different
    key and a different search: those roots are refused instead."""
    prev = -1
    for c in cards:
        if type(c) is not int and not hasattr(c, '__index__'):
            raise TypeError(f'card id {c!r} is not an int')
        c = int(c)
        if not 0 <= c < 90:
            raise ValueError(f'card id {c} outside the deck (0..89): the packed state cannot hold it')
        if c == prev:
            raise ValueError(f'card {c} appears twice in cards: the packed state holds a card set')
        if c < prev:
            raise ValueError(f'cards {tuple(cards)} are not in ascending order (the reference keeps them '
                             'sorted with insort): the packed state would hash a different tuple')
        prev = c


def encode(cards, gems, pts: int, saved: int) -> tuple[int, int]:
    check_cards(cards)
    if len(gems) != COLOR_NUM:
        raise ValueError(f'gems must have {COLOR_NUM} counts: {gems}')
    lo = 0
    hi = 0
    for c in cards:
        if c < 64:
            lo |= 1 << c
        else:
            hi |= 1 << (c - 64)
    for i, g in enumerate(gems):
        if not 0 <= g <= 7:
            raise ValueError(f'gem count out of range: {gems}')
        hi |= g << (26 + 3 * i)
    if not 0 <= pts < 256 or not 0 <= saved < (1 << 15):
        raise ValueError(f'pts/saved out of range: {pts}, {saved}')
    hi |= pts << 41
    hi |= saved << 49
    return lo, hi


def decode(lo: int, hi: int):
    """-> (cards tuple sorted, bonus, gems, pts, saved)."""
    deck = get_deck()
    cards = tuple([c for c in range(64) if lo >> c & 1] + [64 + c for c in range(26) if hi >> c & 1])
    gems = tuple((hi >> (26 + 3 * i)) & 7 for i in range(COLOR_NUM))
    bonus = [0] * COLOR_NUM
    for c in cards:
        bonus[deck[c].bonus.value] += 1
    pts = (hi >> 41) & 0xFF
    saved = hi >> 49
    return cards, tuple(bonus), gems, pts, saved
