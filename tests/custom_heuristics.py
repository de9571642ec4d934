"""User-registered heuristics for the custom-heuristic parity test (HEURISTICS.md:204-229).

Shared by tests/golden/make_golden.py (registered in the reference's HEURISTICS to capture the goldens)
and tests/test_gpu_custom.py (registered in splendor_amd's HEURISTICS).  They read every State field the
reference documents, draw from `random` (so the draw order of `sorted`'s key calls is checked) and return
heavily tied values (so the stability of the prune is checked): one float-valued, one int-valued.
"""
from random import randint


def card_rush(state) -> float:
    return state.pts * 10 + len(state.cards) * 1.5 - sum(state.gems) * 0.25 + randint(1, 4)


def saver(state) -> int:
    return state.pts * 3 + state.saved + max(state.bonus) + randint(0, 2)


CUSTOM = {'card_rush': card_rush, 'saver': saver}
# (goal, name, beam width, seed) of the captured solves
CASES = [(8, 'card_rush', 2000, 0), (10, 'card_rush', 5000, 1), (8, 'saver', 3000, 0), (10, 'saver', 20000, 2)]
