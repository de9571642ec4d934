#!/usr/bin/env python3
"""Time the stable top-k (sb_debug_topk) on random keys: n=41M keep=4M (select + sort) and n=keep=4M
(sort only).  Run under rocprofv3 --kernel-trace for per-kernel times; SPLENDOR_BEAM_LIB picks a variant."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'splendor-rl-gym_amd'))
from splendor_amd.engine import device_topk  # noqa: E402

rng = np.random.default_rng(0)
for n, keep in ((41_000_000, 4_000_000), (4_000_000, 4_000_000)):
    # f64 score images clustered like the heuristics' (few binades, 100 noise steps)
    base = rng.integers(0, 4000, n).astype(np.float64) * 13.37 + 1000.0
    keys = (base + rng.integers(1, 101, n) * 0.01).view(np.uint64)
    for _ in range(3):
        t = time.perf_counter()
        idx = device_topk(keys, keep, 0)
        dt = time.perf_counter() - t
    ref = np.argsort(-keys.view(np.float64), kind='stable')[:keep]
    print(f'n={n} keep={keep}: {dt * 1e3:.1f} ms (incl. copies) exact={np.array_equal(ref, idx)}', flush=True)
