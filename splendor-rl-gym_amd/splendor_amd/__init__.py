"""splendor_amd — MI355X-native beam-search step engine for the Splendor "fastest win" solver.

Drop-in for the per-turn state-expansion hot path of IamJasonBian/Splendor-RL-Gym's
``State.solve`` (src/solver.py:390-464).  The engine is ``libsplendor_beam.so``
(hand-written HIP for gfx950, C-ABI in ``include/splendor_beam.h``); this package is
the host side that keeps the reference's Python interface.
"""
from .deck import COLOR_NUM, MAX_GEMS, Card, Color, get_deck
from .solver import (HEURISTICS, State, aggressive_heuristic, balanced_heuristic, competitive_heuristic,
                     efficiency_heuristic, simple_heuristic)

__all__ = ['COLOR_NUM', 'MAX_GEMS', 'Card', 'Color', 'get_deck', 'HEURISTICS', 'State', 'simple_heuristic',
           'balanced_heuristic', 'aggressive_heuristic', 'efficiency_heuristic', 'competitive_heuristic']
