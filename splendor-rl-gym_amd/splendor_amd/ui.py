"""Terminal rendering of a speedrun solution (same output as the reference's src/ui.py:11-77)."""
from __future__ import annotations

from .deck import Color, get_deck

deck = get_deck()


def format_gems(gems) -> str:
    names = [c.name.title() for c in Color]
    parts = [f'{n}: {k}' for n, k in zip(names, gems) if k > 0]
    return ', '.join(parts) if parts else 'None'


def format_cards(card_indices) -> str:
    if not card_indices:
        return 'None'
    return ', '.join(str(deck[i]) for i in card_indices)


def format_state(state, step: int) -> str:
    return '\n'.join([
        f'\n=== Step {step} ===',
        f'Points: {state.pts}',
        f'Gems Saved: {state.saved}',
        f'Held Gems: {format_gems(state.gems)}',
        f'Bonus Gems: {format_gems(state.bonus)}',
        f'Cards: {format_cards(state.cards)}',
    ])


def render_solution(solution) -> None:
    print('\n' + '=' * 60)
    print('SOLUTION PATH')
    print('=' * 60)
    for step, state in enumerate(solution):
        print(format_state(state, step))
    final = solution[-1]
    print('\n' + '=' * 60)
    print(f'FINAL: {final.pts} points in {len(solution) - 1} moves')
    print('=' * 60)
