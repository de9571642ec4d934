"""Python handle over one HIP beam engine (``sb_engine``): the device side of ``State.solve``."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

HEURISTIC_IDS = {'simple': 0, 'balanced': 1, 'aggressive': 2, 'efficiency': 3,
                 # on a speedrun State, competitive_heuristic returns balanced_heuristic (src/solver.py:289-296)
                 'competitive': 1}


class BeamEngine:
    """Stepwise speedrun beam search on one MI355X (one iteration of src/solver.py:434-457 per step)."""

    def __init__(self, *, goal_pts: int, use_heuristic: bool, heuristic: int, beam_width: int,
                 mt_state625, root_lo: int = 0, root_hi: int = 0, device: int = 0, visited_log2: int = 0,
                 timing: bool = False, test_flags: int = 0):
        L.ensure_tables()
        # test_flags: sb_config.flags bits 2-4 (include/splendor_beam.h): alternative select paths, eager growth
        cfg = L.SbConfig(goal_pts=int(goal_pts), use_heuristic=int(bool(use_heuristic)), heuristic=int(heuristic),
                         device=int(device), beam_width=int(beam_width), visited_log2=int(visited_log2),
                         flags=(1 if timing else 0) | (int(test_flags) & 28), world_size=1, rank=0)
        st = np.ascontiguousarray(np.array(mt_state625, dtype=np.uint32))
        if st.shape != (625,):
            raise ValueError('mt_state625 must be random.getstate()[1] (625 words)')
        h = C.c_void_p()
        L.check(L.lib().sb_create(C.byref(cfg), st, int(root_lo), int(root_hi), C.byref(h)), 'sb_create')
        self._h = h
        self.done = False
        self.turn = 0
        self.host_scored = bool(use_heuristic) and int(heuristic) == L.SB_HEUR_HOST
        self.pending = 0

    def close(self):
        if getattr(self, '_h', None):
            L.lib().sb_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def step(self) -> dict:
        s = L.SbStepStats()
        L.check(L.lib().sb_step(self._h, C.byref(s)), 'sb_step')
        d = s.as_dict()
        self.done = d['done']
        if not self.done:
            self.turn += 1
        self.pending = d['n_unique'] if (self.host_scored and not self.done) else 0
        return d

    def read_next(self, start: int = 0, n: int | None = None):
        """next_queue of a host-scored turn (heuristic=SB_HEUR_HOST) after step(): packed (lo, hi) arrays."""
        if n is None:
            n = self.pending - start
        lo = np.zeros(n, np.uint64)
        hi = np.zeros(n, np.uint64)
        L.check(L.lib().sb_read_next(self._h, int(start), int(n), lo.ctypes.data, hi.ctypes.data), 'sb_read_next')
        return lo, hi

    def prune(self, scores) -> int:
        """Stable descending top-k of host scores over next_queue (sorted(..., reverse=True)[:beam_width]) on the
        device; the next turn's beam is written and its expansion launched.  Returns the kept count."""
        sc = np.ascontiguousarray(np.asarray(scores, dtype=np.float64))
        kept = C.c_int64()
        L.check(L.lib().sb_prune(self._h, sc.ctypes.data, len(sc), C.byref(kept)), 'sb_prune')
        self.pending = 0
        return kept.value

    def turn_times(self, t: int) -> dict:
        """Device phase times (ms) of completed turn t (engine created with timing=True)."""
        out = np.zeros(7, np.float32)
        L.check(L.lib().sb_turn_times(self._h, int(t), out), 'sb_turn_times')
        return dict(zip(('ms_expand', 'ms_survive', 'ms_mt', 'ms_emit', 'ms_select', 'ms_gather', 'ms_total'),
                        (float(x) for x in out)))

    def num_turns(self) -> int:
        n = C.c_int32()
        L.check(L.lib().sb_num_turns(self._h, C.byref(n)))
        return n.value

    def turn_size(self, t: int) -> int:
        n = C.c_int64()
        L.check(L.lib().sb_turn_size(self._h, int(t), C.byref(n)), 'sb_turn_size')
        return n.value

    def read_turn(self, t: int, start: int = 0, n: int | None = None, *, keys: bool = True):
        size = self.turn_size(t)
        if n is None:
            n = size - start
        lo = np.zeros(n, np.uint64)
        hi = np.zeros(n, np.uint64)
        par = np.zeros(n, np.uint32)
        key = np.zeros(n, np.uint64) if keys else None
        L.check(L.lib().sb_read_turn(self._h, int(t), int(start), int(n), lo.ctypes.data, hi.ctypes.data,
                                     par.ctypes.data, key.ctypes.data if keys else None), 'sb_read_turn')
        return lo, hi, par, key

    def state_at(self, t: int, rank: int):
        lo, hi, _, _ = self.read_turn(t, rank, 1, keys=False)
        return int(lo[0]), int(hi[0])

    def path(self):
        cap = self.num_turns()
        lo = np.zeros(cap, np.uint64)
        hi = np.zeros(cap, np.uint64)
        n = C.c_int32()
        L.check(L.lib().sb_path(self._h, lo, hi, cap, C.byref(n)), 'sb_path')
        return [(int(lo[i]), int(hi[i])) for i in range(n.value)]

    def mt_state(self) -> np.ndarray:
        out = np.zeros(625, np.uint32)
        L.check(L.lib().sb_get_mt_state(self._h, out), 'sb_get_mt_state')
        return out

    def sync(self):
        L.check(L.lib().sb_sync(self._h), 'sb_sync')

    def sync_engine(self):
        """Wait for the launched turns (engine stream), not for noise generation running ahead."""
        L.check(L.lib().sb_sync_engine(self._h), 'sb_sync_engine')

    def set_lookahead(self, on):
        """Launch the next turn's expansion at the end of step() (default) or at the start of the next."""
        L.check(L.lib().sb_set_lookahead(self._h, int(bool(on))), 'sb_set_lookahead')

    def visited_size(self) -> int:
        v = C.c_uint64()
        L.check(L.lib().sb_visited_size(self._h, C.byref(v)))
        return v.value

    def visited_capacity(self) -> tuple[int, int]:
        """(slots, rebuilds): the visited set grows between turns (include/splendor_beam.h)."""
        return L.visited_capacity(self._h)

    def visited_stats(self) -> dict:
        """Growth record of the visited set (sb_visited_stats): rebuilds short of the worst case or skipped, peak load."""
        return L.visited_stats(self._h)


def device_successors(lo, hi, device: int = 0):
    """Ordered successors of a batch of packed states on the GPU (the k_expand enumeration)."""
    L.ensure_tables()
    lo = np.ascontiguousarray(np.asarray(lo, dtype=np.uint64))
    hi = np.ascontiguousarray(np.asarray(hi, dtype=np.uint64))
    n = len(lo)
    olo = np.zeros(n * 192, np.uint64)
    ohi = np.zeros(n * 192, np.uint64)
    okey = np.zeros(n * 192, np.uint64)
    cnt = np.zeros(n, np.int32)
    L.check(L.lib().sb_debug_successors(device, lo, hi, n, olo, ohi, okey, cnt), 'sb_debug_successors')
    return [(olo[i * 192:i * 192 + cnt[i]], ohi[i * 192:i * 192 + cnt[i]], okey[i * 192:i * 192 + cnt[i]])
            for i in range(n)]


def device_mt_words(state625, n: int, device: int = 0, producers: int | None = None,
                    twists: int = 1) -> np.ndarray:
    """Tempered MT19937 words from the device jump-ahead producers (continuing from state625)."""
    out = np.zeros(n, np.uint32)
    st = np.ascontiguousarray(np.array(state625, np.uint32))
    if producers is None:
        L.check(L.lib().sb_debug_mt_words(device, st, n, out), 'sb_debug_mt_words')
    else:
        L.check(L.lib().sb_debug_mt_words_cfg(device, st, n, producers, twists, out), 'sb_debug_mt_words_cfg')
    return out


def device_scores(heuristic: int, lo, hi, k, device: int = 0) -> np.ndarray:
    L.ensure_tables()
    lo = np.ascontiguousarray(np.asarray(lo, dtype=np.uint64))
    hi = np.ascontiguousarray(np.asarray(hi, dtype=np.uint64))
    k = np.ascontiguousarray(np.asarray(k, dtype=np.int32))
    out = np.zeros(len(lo), np.float64)
    L.check(L.lib().sb_debug_scores(device, heuristic, lo, hi, k, len(lo), out), 'sb_debug_scores')
    return out


def device_topk(keys, keep: int, device: int = 0) -> np.ndarray:
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64))
    m = min(len(keys), keep)
    out = np.zeros(m, np.uint32)
    L.check(L.lib().sb_debug_topk(device, keys, len(keys), keep, out), 'sb_debug_topk')
    return out
