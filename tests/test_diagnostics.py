"""Failure messages that must be readable from one run, checked on CPU.

* Every engine device allocation goes through one allocator (csrc/sb_engine.hip dev_malloc) whose failure names
  what was being allocated, the bytes requested and the HBM free at that moment — the visited-set rebuild of
  gpurun_out/r4oe/c5.log:159 failed with a bare `hipMalloc ... out of memory`.  SB_DEBUG_HBM_LIMIT forces the
  failure without a GPU.
* The C5 world-8 tests wait for the previous test's ranks to hand their HBM back; when it does not come back,
  the wait fails the test as a precondition with the free and needed GiB instead of returning silently.
"""
import os
import subprocess
import sys

import pytest

from conftest import REPO

_PROBE = r'''
import sys
sys.path.insert(0, sys.argv[1])
from splendor_amd import _lib
L = _lib.lib()
rc = L.sb_debug_alloc(1 << 30)
print(rc)
print(L.sb_last_error().decode())
'''


def test_engine_allocation_failure_names_bytes_and_free_hbm():
    env = dict(os.environ, SB_DEBUG_HBM_LIMIT=str(1 << 20))
    out = subprocess.run([sys.executable, '-c', _PROBE, os.path.join(REPO, 'splendor-rl-gym_amd')], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    rc, msg = out.stdout.strip().split('\n', 1)
    assert int(rc) == -4   # SB_ERR_CAPACITY: out of memory
    assert 'sb_debug_alloc' in msg and '1073741824 bytes' in msg and '1.000 GiB' in msg, msg
    assert 'free HBM' in msg and 'SB_DEBUG_HBM_LIMIT=1048576' in msg, msg


def test_wait_device_memory_fails_loudly_on_timeout():
    from test_gpu_big import _wait_device_memory
    fake = lambda: (3 * 2**30, 288 * 2**30)
    with pytest.raises(pytest.fail.Exception) as ei:
        _wait_device_memory(min_free_gib=240.0, timeout_s=0.2, mem_get_info=fake)
    assert '3.0 GiB free' in str(ei.value) and '240.0 GiB needed' in str(ei.value)
    assert _wait_device_memory(min_free_gib=2.0, timeout_s=0.2, mem_get_info=fake) == 3 * 2**30
