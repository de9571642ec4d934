"""Realistic-mode engine handle (sbr_* entry points) and MultiPlayerState.solve (src/solver.py:750-860)."""
from __future__ import annotations

import ctypes as C
import random

import numpy as np

from . import _lib as L
from .realistic import RW, game_params, pack_state, unpack_state


def _bind():
    lib = L.lib()
    if getattr(lib, '_sbr_bound', False):
        return lib
    vp = C.c_void_p
    i32p = np.ctypeslib.ndpointer(np.int32, flags='C')
    u32p = np.ctypeslib.ndpointer(np.uint32, flags='C')
    u64p = np.ctypeslib.ndpointer(np.uint64, flags='C')
    lib.sbr_create.argtypes = [C.POINTER(L.SbConfig), i32p, i32p, u32p, u64p, C.POINTER(vp)]
    lib.sbr_step.argtypes = [vp, C.POINTER(L.SbStepStats)]
    lib.sbr_read_turn.argtypes = [vp, C.c_int32, C.c_int64, C.c_int64, vp, vp, vp]
    lib.sbr_path.argtypes = [vp, u64p, C.c_int32, C.POINTER(C.c_int32)]
    lib._sbr_bound = True
    return lib


def device_tiers(state):
    """Tier lists for the device: 4 placeholder slots + the remaining deck (deck pointer 0 at the root)."""
    m = state.market
    return [[0, 0, 0, 0] + list(m.tier1_deck), [0, 0, 0, 0] + list(m.tier2_deck), [0, 0, 0, 0] + list(m.tier3_deck)]


class RealisticEngine:
    """Stepwise realistic beam search on one MI355X."""

    def __init__(self, root, *, beam_width: int, mt_state625, device: int = 0, visited_log2: int = 0, tiers=None,
                 timing: bool = False):
        L.ensure_tables()
        lib = _bind()
        self.config = root.config
        self.tiers0 = tiers if tiers is not None else device_tiers(root)
        self.params, self.tiers = game_params(root.config, self.tiers0)
        cfg = L.SbConfig(goal_pts=root.config.target_points, use_heuristic=1, heuristic=0, device=int(device),
                         beam_width=int(beam_width), visited_log2=int(visited_log2), flags=1 if timing else 0,
                         world_size=1, rank=0)
        h = C.c_void_p()
        st = np.ascontiguousarray(np.array(mt_state625, dtype=np.uint32))
        L.check(lib.sbr_create(C.byref(cfg), self.params, self.tiers, st, pack_state(root, self.tiers0), C.byref(h)),
                'sbr_create')
        self._h = h
        self.done = False

    def close(self):
        if getattr(self, '_h', None):
            L.lib().sb_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def step(self) -> dict:
        s = L.SbStepStats()
        L.check(_bind().sbr_step(self._h, C.byref(s)), 'sbr_step')
        d = s.as_dict()
        self.done = d['done']
        return d

    def turn_times(self, t: int) -> dict:
        """Device phase times (ms) of completed turn t (engine created with timing=True): expansion
        (k_rexpand), survivor count + scan, emission, top-k, gather, total."""
        out = np.zeros(7, np.float32)
        L.check(L.lib().sb_turn_times(self._h, int(t), out), 'sb_turn_times')
        return dict(zip(('ms_expand', 'ms_survive', 'ms_mt', 'ms_emit', 'ms_select', 'ms_gather', 'ms_total'),
                        (float(x) for x in out)))

    def num_turns(self) -> int:
        n = C.c_int32()
        L.check(L.lib().sb_num_turns(self._h, C.byref(n)))
        return n.value

    def turn_size(self, t) -> int:
        n = C.c_int64()
        L.check(L.lib().sb_turn_size(self._h, int(t), C.byref(n)))
        return n.value

    def read_turn(self, t, start=0, n=None, *, keys=True):
        size = self.turn_size(t)
        n = size - start if n is None else n
        w = np.zeros(n * RW, np.uint64)
        par = np.zeros(n, np.uint32)
        key = np.zeros(n, np.uint64) if keys else None
        L.check(_bind().sbr_read_turn(self._h, int(t), int(start), int(n), w.ctypes.data, par.ctypes.data,
                                      key.ctypes.data if keys else None), 'sbr_read_turn')
        return w.reshape(n, RW), par, key

    def state_at(self, t, rank):
        w, _, _ = self.read_turn(t, rank, 1, keys=False)
        return unpack_state(w[0], self.config, self.tiers0, t)

    def path_words(self):
        cap = self.num_turns()
        w = np.zeros(cap * RW, np.uint64)
        n = C.c_int32()
        L.check(_bind().sbr_path(self._h, w, cap, C.byref(n)), 'sbr_path')
        return w[:n.value * RW].reshape(n.value, RW)

    def path(self):
        return [unpack_state(w, self.config, self.tiers0, t) for t, w in enumerate(self.path_words())]

    def visited_capacity(self) -> tuple[int, int]:
        """(slots, rebuilds) of the visited set (grown between turns)."""
        return L.visited_capacity(self._h)

    def visited_stats(self) -> dict:
        return L.visited_stats(self._h)

    def mt_state(self):
        out = np.zeros(625, np.uint32)
        L.check(L.lib().sb_get_mt_state(self._h, out))
        return out


def solve_realistic(root, *, beam_width=20_000, verbose=True, device=0, tiers=None, heuristic_name='competitive',
                    sync_random=True):
    """MultiPlayerState.solve: same banner, progress lines and result as the reference (src/solver.py:750-860)."""
    cfg = root.config
    if verbose:
        print('=' * 60)
        print('REALISTIC MODE SOLVER')
        print('=' * 60)
        print(f'Target Points: {cfg.target_points}')
        print(f'Number of Players: {cfg.num_players}')
        print(f'Gems per Color: {cfg.gems_per_color}')
        print(f'Heuristic: {heuristic_name}')
        print(f'Beam Width: {beam_width:,}')
        print('Card Visibility: 12 cards (4 per tier)')
        shuffled = root.market.tier1_deck != root.market.tier1_deck[:1]
        print(f'Market Shuffled: {"Yes" if shuffled else "No (deterministic)"}')
        print('=' * 60)
        print()
    if cfg.num_players != 2 and cfg.num_players not in (3, 4):
        raise ValueError('players must be 2..4')
    st = random.getstate()
    eng = RealisticEngine(root, beam_width=beam_width, mt_state625=st[1], device=device, tiers=tiers)
    try:
        turn = 0
        while True:
            if verbose and turn % 100 == 0:
                print(f'turn={turn:<10} Queue size: {eng.turn_size(turn)}')
            s = eng.step()
            if verbose:
                for rank, pts in s['records']:
                    print(f'max_pts={pts:<7} {eng.state_at(turn, rank)}')
            if s['done']:
                if s['n_unique'] > 0:   # stopped by the 1000-turn cap, not by game over / empty queue
                    print('Warning: Reached turn limit (1000)')
                break
            turn += 1
        path = eng.path()
        if sync_random:
            mt = eng.mt_state()
            random.setstate((st[0], tuple(int(x) for x in mt), st[2]))
    finally:
        eng.close()
    return path
