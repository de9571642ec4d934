"""The C-ABI library builds for gfx950, loads without a GPU and exports every symbol the header declares."""
import ctypes
import os
import re
import subprocess

from conftest import REPO
from splendor_amd import _lib

HEADER = os.path.join(REPO, 'include', 'splendor_beam.h')


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char\*)\s+(sb[dr]?_\w+)\s*\(', text, re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    assert set(_lib.EXPORTED) == set(syms), set(_lib.EXPORTED) ^ set(syms)


def test_library_loads_and_exports_all_symbols():
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert L.sb_version() >= 1
    out = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True, text=True).stdout
    for s in declared_symbols():
        assert re.search(rf'\bT {s}$', out, re.M), s


def test_library_targets_gfx950():
    out = subprocess.run(['strings', _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert 'gfx950' in out


def test_argument_errors_without_gpu():
    """Null handles/args are rejected with an error code before any device work."""
    L = _lib.lib()
    assert L.sb_step(None, None) == _lib.SB_ERR_ARG
    assert L.sb_sync(None) == _lib.SB_ERR_ARG
    assert L.sb_read_next(None, 0, 0, None, None) == _lib.SB_ERR_STATE
    assert L.sb_prune(None, None, 0, None) == _lib.SB_ERR_ARG
    cfg = _lib.SbConfig(goal_pts=3, use_heuristic=0, heuristic=0, device=0, beam_width=0)
    import numpy as np
    h = ctypes.c_void_p()
    _lib.ensure_tables()
    rc = L.sb_create(ctypes.byref(cfg), np.zeros(625, np.uint32), 0, 0, ctypes.byref(h))
    assert rc == _lib.SB_ERR_ARG
    assert b'beam_width' in L.sb_last_error()


def test_init_tables_validates_deck():
    import numpy as np
    L = _lib.lib()
    bad = np.zeros(90 * 7, np.int32)
    bad[0] = 9
    rc = L.sb_init_tables(bad, np.zeros(11 * 256), np.zeros(100))
    assert rc == _lib.SB_ERR_ARG
    _lib._tables_ready = False
    _lib.ensure_tables()


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A library built from other sources than the tree's is refused: the build
    stamps sb_build_id with the sources' sha256; editing any source changes the tree's hash."""
    import shutil
    L = _lib.lib()
    _lib.check_fresh(L, _lib.LIB_PATH)          # the in-tree build matches its sources
    csrc = tmp_path / 'csrc'
    shutil.copytree(_lib.CSRC, csrc)
    monkeypatch.setattr(_lib, 'CSRC', str(csrc))
    assert _lib.source_hash() == L.sb_build_id().decode()
    with open(csrc / 'sb_engine.hip', 'a') as f:  # "touch" with an edit
        f.write('\n// edited\n')
    assert _lib.source_hash() != L.sb_build_id().decode()
    import pytest
    with pytest.raises(ImportError, match='stale'):
        _lib.check_fresh(L, _lib.LIB_PATH)


def test_sharded_slice_capacity_is_checked():
    """Sharded own-claim tags hold a rank's local parent rank in 26 bits: a beam whose slice
    per rank exceeds 2^26 is refused at sb_create (and a larger slice at sbd_expand_launch)."""
    import numpy as np
    L = _lib.lib()
    _lib.ensure_tables()
    h = ctypes.c_void_p()
    cfg = _lib.SbConfig(goal_pts=15, use_heuristic=1, heuristic=3, device=0, beam_width=(1 << 27) + 2,
                        world_size=2, rank=0)
    rc = L.sb_create(ctypes.byref(cfg), np.zeros(625, np.uint32), 0, 0, ctypes.byref(h))
    assert rc == _lib.SB_ERR_CAPACITY
    assert b'2^26' in L.sb_last_error()


def test_sharded_entry_points_refuse_a_null_engine():
    """Every sharded entry point (sbd_*) the header declares answers a null engine with SB_ERR_ARG before
    touching the device: arguments typed from the header's own parameter lists, all zero / null."""
    _lib.lib()
    L = ctypes.CDLL(_lib.LIB_PATH)   # fresh function objects: no argtypes another test's backend may have set
    text = open(HEADER).read()
    probed = 0
    for m in re.finditer(r'^\s*int\s+(sbd_\w+)\s*\(([^)]*)\)\s*;', text, re.M):
        name, params = m.group(1), [p.strip() for p in m.group(2).split(',')]
        args = [ctypes.c_void_p(None) if '*' in p else ctypes.c_int64(0) if 'int64' in p else ctypes.c_int32(0)
                for p in params]
        f = getattr(L, name)
        f.restype = ctypes.c_int
        assert f(*args) == _lib.SB_ERR_ARG, name
        probed += 1
    assert probed == len([s for s in declared_symbols() if s.startswith('sbd_')])
