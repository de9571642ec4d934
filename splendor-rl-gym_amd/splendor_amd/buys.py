"""Possible-buys table and its on-disk formats (flag compatibility with src/buys.py:8-49).

The engine tests affordability directly on the device (cost <= gems + bonus), so it needs no table;
`-b` / `-e` keep the reference's buys.pickle / buys.txt outputs for users who rely on them.
"""
from __future__ import annotations

import pickle
from itertools import product
from pathlib import Path

from .deck import COLOR_NUM, MAX_GEMS, get_deck

BUYS_PATH = Path('buys.pickle')


def possible_buys() -> dict:
    deck = get_deck()
    out = {}
    for g in product(range(MAX_GEMS + 1), repeat=COLOR_NUM):
        out[g] = tuple(c.index for c in deck if all(x <= y for x, y in zip(c.cost, g)))
    return out


def store_buys(buys: dict, path: Path = BUYS_PATH) -> None:
    with path.open('wb') as f:
        pickle.dump(buys, f, pickle.HIGHEST_PROTOCOL)


def load_buys(*, update: bool = False, path: Path = BUYS_PATH) -> dict:
    if not path.exists() or update:
        print('Generating buys...')
        buys = possible_buys()
        print('Pickling buys...')
        store_buys(buys, path)
        print('Pickling finished.')
        return buys
    with path.open('rb') as f:   # our own file, written by store_buys
        print('Unpickling buys...')
        return pickle.load(f)


def export_buys_to_txt(path: Path = Path('buys.txt')) -> None:
    buys = possible_buys()
    with path.open('w', encoding='utf-8') as f:
        print('Writing buys to a text file...')
        for g, b in buys.items():
            f.write(f'{g}: {b}\n')
