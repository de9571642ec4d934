"""ctypes binding of ``libsplendor_beam.so`` (declared in ``include/splendor_beam.h``).

The product path has exactly one implementation: the HIP engine.  If the shared
library is missing or the GPU is unavailable, every entry point raises — there is
no CPU fallback (the CPU restatement under ``oracle/`` is test infrastructure).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(PKG_DIR), 'csrc')
LIB_PATH = os.path.join(PKG_DIR, 'libsplendor_beam.so')
# developer knob: load a differently tuned build of the same sources (profiles/variants.sh)
LOAD_PATH = os.environ.get('SPLENDOR_BEAM_LIB', LIB_PATH)
SOURCES = ['sb_engine.hip', 'sb_scan.hip', 'sb_sort.hip', 'sb_mt.hip', 'sb_gf2.hip']

SB_OK = 0
SB_ERR_ARG = -1
SB_ERR_HIP = -2
SB_ERR_STATE = -3
SB_ERR_CAPACITY = -4
SB_ERR_NOTABLES = -5
SB_HEUR_HOST = 15   # a Python HEURISTICS callable scores next_queue on the host (sb_read_next / sb_prune)

# exponents of the host-captured pow tables, in SB row order (include/splendor_beam.h)
POW_EXPONENTS = (0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 1.2, 2.0, 2.5, 2.8, 3.2)
POW_BASES = 256
EXPORTED = ('sb_init_tables', 'sb_create', 'sb_step', 'sb_read_next', 'sb_prune', 'sb_turn_times', 'sb_num_turns', 'sb_turn_size', 'sb_read_turn', 'sb_path',
            'sb_get_mt_state', 'sb_sync', 'sb_set_lookahead', 'sb_sync_engine', 'sb_visited_size', 'sb_visited_capacity', 'sb_visited_stats', 'sb_destroy', 'sb_last_error', 'sb_version', 'sb_build_id',
            'sb_debug_successors', 'sb_debug_alloc', 'sb_debug_mt_words', 'sb_debug_mt_words_cfg', 'sb_debug_scores', 'sb_debug_topk', 'sb_debug_topk_scores', 'sb_debug_expand_bench', 'sb_debug_oe_merge',
            'sbd_goal_table', 'sbd_expand_launch', 'sbd_expand_counts', 'sbd_expand_parts', 'sbd_part_counts', 'sbd_part_pack', 'sbd_send_buffer', 'sbd_set_claim_stream', 'sbd_owner_total', 'sbd_grow_receive', 'sbd_expand_defer', 'sbd_raw_total', 'sbd_pack', 'sbd_owner_begin', 'sbd_owner_claim', 'sbd_owner_finish', 'sbd_owner_claim_all', 'sbd_owner_claim_part', 'sbd_pack_bits', 'sbd_unpack_bits', 'sbd_pack_bits_segs', 'sbd_unpack_bits_segs', 'sbd_apply', 'sbd_apply_finish', 'sbd_emit',
            'sbd_key_range', 'sbd_sel_begin', 'sbd_sel_begin_approx', 'sbd_sel_hist', 'sbd_sel_pick', 'sbd_sel_compact', 'sbd_sel_eq', 'sbd_set_stream', 'sbd_noise_info', 'sbd_noise_chunk', 'sbd_noise_sync', 'sbd_noise_pack', 'sbd_noise_fill', 'sbd_noise_fill_ranges', 'sbd_partition', 'sbd_partition_bfs', 'sbd_block_counts', 'sbd_sel_eq_blocks', 'sbd_partition_blocks', 'sbd_dest_subcounts', 'sbd_pack_kept', 'sbd_pack_kept_grouped', 'sbd_unpack_kept', 'sbd_receive', 'sbd_mark_done',
            'sbd_mig_launch', 'sbd_mig_counts', 'sbd_mig_pack', 'sbd_mig_expand', 'sbd_mig_claim', 'sbd_mig_apply', 'sbd_mig_place', 'sbd_keypass_ms',
            'sbd_oe_pack', 'sbd_oe_counts', 'sbd_oe_emit', 'sbd_oe_ties', 'sbd_oe_tie_read', 'sbd_oe_partition',
            'sbd_oe_partition_bfs', 'sbd_oe_segments',
            'sbr_create', 'sbr_step', 'sbr_read_turn', 'sbr_path')


class SplendorBeamError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f'[{code}] {msg}')
        self.code = code


class SbConfig(C.Structure):
    _fields_ = [('goal_pts', C.c_int32), ('use_heuristic', C.c_int32), ('heuristic', C.c_int32),
                ('device', C.c_int32), ('beam_width', C.c_int64), ('visited_log2', C.c_int32),
                ('flags', C.c_int32), ('world_size', C.c_int32), ('rank', C.c_int32)]


class SbStepStats(C.Structure):
    _fields_ = [('n_parents', C.c_int64), ('n_raw', C.c_int64), ('n_unique', C.c_int64), ('n_kept', C.c_int64),
                ('done', C.c_int32), ('turn', C.c_int32), ('winner_rank', C.c_int64), ('n_records', C.c_int32),
                ('record_pts', C.c_int32 * 32), ('record_rank', C.c_int64 * 32), ('noise_draws', C.c_uint64),
                ('ms_expand', C.c_float), ('ms_survive', C.c_float), ('ms_emit', C.c_float),
                ('ms_select', C.c_float), ('ms_sort', C.c_float), ('ms_gather', C.c_float), ('ms_mt', C.c_float),
                ('ms_total', C.c_float)]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_ if f not in ('record_pts', 'record_rank')}
        d['records'] = [(self.record_rank[i], self.record_pts[i]) for i in range(self.n_records)]
        d['done'] = bool(self.done)
        return d


HEADER = os.path.join(os.path.dirname(os.path.dirname(PKG_DIR)), 'include', 'splendor_beam.h')


def source_hash() -> str | None:
    """sha256 prefix over the engine's sources (csrc/*.hip, *.inc, *.h and the C-ABI header), or None
    when the sources are not present (an installed library without its tree)."""
    if not os.path.isdir(CSRC):
        return None
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith(('.hip', '.inc', '.h')))
    for f in files:
        h.update(f.encode() + b'\0')
        with open(os.path.join(CSRC, f), 'rb') as fh:
            h.update(fh.read())
    if os.path.exists(HEADER):
        with open(HEADER, 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build(verbose: bool = False, out: str | None = None, defines: tuple = ()) -> str:
    """Compile the HIP sources for gfx950 into the in-tree shared library (or `out`, with -D `defines`)."""
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    out = out or LIB_PATH
    cmd = ['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off',
           '-Wall', '-Wno-unused-function', f'-DSB_BUILD_ID="{source_hash()}"', *[f'-D{d}' for d in defines], *srcs,
           '-o', out]
    if verbose:
        print(' '.join(cmd))
    subprocess.run(cmd, check=True)
    return out


def check_fresh(L, path: str) -> None:
    """Refuse a library built from other sources than the tree's (a run that skipped build())."""
    want = source_hash()
    L.sb_build_id.restype = C.c_char_p
    have = L.sb_build_id().decode()
    if want is not None and have != want:
        raise ImportError(f'{path} is stale: built from sources {have}, tree is {want}; '
                          'rebuild it (python __graft_entry__.py, or splendor_amd._lib.build())')


_lib = None
_tables_ready = False


def lib():
    """Load (never silently replace) the engine library."""
    global _lib
    if _lib is None:
        if not os.path.exists(LOAD_PATH):
            raise ImportError(f'{LOAD_PATH} missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)')
        L = C.CDLL(LOAD_PATH)
        check_fresh(L, LOAD_PATH)
        u64p = np.ctypeslib.ndpointer(np.uint64, flags='C')
        u32p = np.ctypeslib.ndpointer(np.uint32, flags='C')
        i32p = np.ctypeslib.ndpointer(np.int32, flags='C')
        f64p = np.ctypeslib.ndpointer(np.float64, flags='C')
        vp = C.c_void_p
        L.sb_init_tables.argtypes = [i32p, f64p, f64p]
        L.sb_create.argtypes = [C.POINTER(SbConfig), u32p, C.c_uint64, C.c_uint64, C.POINTER(vp)]
        L.sb_step.argtypes = [vp, C.POINTER(SbStepStats)]
        L.sb_read_next.argtypes = [vp, C.c_int64, C.c_int64, vp, vp]
        L.sb_prune.argtypes = [vp, vp, C.c_int64, C.POINTER(C.c_int64)]
        L.sb_turn_times.argtypes = [vp, C.c_int32, np.ctypeslib.ndpointer(np.float32, flags='C')]
        L.sb_num_turns.argtypes = [vp, C.POINTER(C.c_int32)]
        L.sb_turn_size.argtypes = [vp, C.c_int32, C.POINTER(C.c_int64)]
        L.sb_read_turn.argtypes = [vp, C.c_int32, C.c_int64, C.c_int64, vp, vp, vp, vp]
        L.sb_path.argtypes = [vp, u64p, u64p, C.c_int32, C.POINTER(C.c_int32)]
        L.sb_get_mt_state.argtypes = [vp, u32p]
        L.sb_visited_size.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.sb_visited_capacity.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]
        L.sb_visited_stats.argtypes = [vp, vp]
        L.sb_sync.argtypes = [vp]
        L.sb_set_lookahead.argtypes = [vp, C.c_int32]
        L.sb_sync_engine.argtypes = [vp]
        L.sb_destroy.argtypes = [vp]
        L.sb_destroy.restype = None
        L.sb_last_error.restype = C.c_char_p
        L.sb_debug_alloc.argtypes = [C.c_uint64]
        L.sb_debug_successors.argtypes = [C.c_int32, u64p, u64p, C.c_int64, u64p, u64p, u64p, i32p]
        L.sb_debug_mt_words.argtypes = [C.c_int32, u32p, C.c_int64, u32p]
        L.sb_debug_mt_words_cfg.argtypes = [C.c_int32, u32p, C.c_int64, C.c_int32, C.c_int64, u32p]
        L.sb_debug_scores.argtypes = [C.c_int32, C.c_int32, u64p, u64p, i32p, C.c_int64, f64p]
        L.sb_debug_topk.argtypes = [C.c_int32, u64p, C.c_int64, C.c_int64, u32p]
        L.sb_debug_topk_scores.argtypes = [C.c_int32, f64p, C.c_int64, C.c_int64, u32p]
        L.sb_debug_oe_merge.argtypes = [C.c_int32, u32p, C.c_int64, C.c_int32,
                                        np.ctypeslib.ndpointer(np.int64, flags='C'), u32p]
        _lib = L
    return _lib


def visited_capacity(h) -> tuple[int, int]:
    """(slots, rebuilds) of a handle's visited set (sb_visited_capacity)."""
    cap, n = C.c_uint64(), C.c_int32()
    check(lib().sb_visited_capacity(h, C.byref(cap), C.byref(n)), 'sb_visited_capacity')
    return cap.value, n.value


def visited_stats(h) -> dict:
    """The visited set's growth record (sb_visited_stats): slots, rebuilds, rebuilds that fell short of the turn's worst
    case (free HBM), rebuilds wanted and not made, the peak load after a turn, keys."""
    import numpy as np
    out = np.zeros(6, np.uint64)
    check(lib().sb_visited_stats(h, out.ctypes.data), 'sb_visited_stats')
    return {'slots': int(out[0]), 'rebuilds': int(out[1]), 'rebuilds_short': int(out[2]), 'rebuilds_skipped': int(out[3]),
            'peak_load': round(int(out[4]) * 1e-6, 6), 'keys': int(out[5])}


def check(rc: int, what: str = ''):
    if rc != SB_OK:
        msg = lib().sb_last_error().decode(errors='replace')
        raise SplendorBeamError(rc, f'{what}: {msg}' if what else msg)


def pow_tables() -> np.ndarray:
    """float(x) ** e for the heuristics' exponents — Python's own float pow (libm), captured exactly."""
    t = np.empty((len(POW_EXPONENTS), POW_BASES), dtype=np.float64)
    for r, e in enumerate(POW_EXPONENTS):
        for x in range(POW_BASES):
            t[r, x] = x ** e
    return t


def noise_table() -> np.ndarray:
    """randint(1, 100) * 0.01 for k = 1..100 (src/solver.py:215)."""
    return np.array([k * 0.01 for k in range(1, 101)], dtype=np.float64)


def ensure_tables():
    global _tables_ready
    if not _tables_ready:
        from .deck import deck_rows
        check(lib().sb_init_tables(np.array(deck_rows(), dtype=np.int32), np.ascontiguousarray(pow_tables().ravel()),
                                   noise_table()), 'sb_init_tables')
        _tables_ready = True
