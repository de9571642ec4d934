"""Visited-set claim protocol under contention (GPU, through the C-ABI sbd_owner_* entry points).

The owner-side claim (csrc/sb_dist.inc claim_rec over probe_insert, csrc/sb_engine.hip) must settle
every key to its first occurrence in record-index order — `if next_step in trail: continue` with
first-occurrence order, src/solver.py:446-450 — however the claims interleave: heavy duplication
(thousands of records per key, many lanes of one wave on one slot), long probe chains (table at
~50% load) and chunks claimed out of index order (later chunks first, so earlier records displace
holders and mark them lost).  Expected answers come from numpy: ret[i] = 1 iff i is the first index
of keys[i].
"""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _backend(log2):
    """Owner rank 0 of a world of 2: every record comes from source rank 1 (a rank's own children never
    become records, sbd_expand claims them itself)."""
    from splendor_amd.dist import HipBackend
    random.seed(0)
    return HipBackend(rank=0, world=2, device_index=0, goal_pts=15, use_heuristic=False, heuristic=0,
                      beam_width=1000, mt_state625=random.getstate()[1], visited_log2=log2)


def _keys(rng, n_heavy, heavy_pool, n_light, light_pool):
    from splendor_amd.codec import state_key
    root = np.uint64(state_key((), (0, 0, 0, 0, 0)) & (2**64 - 1))
    pool_h = rng.integers(1, 2**63, size=heavy_pool, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    pool_l = rng.integers(1, 2**63, size=light_pool, dtype=np.uint64) * np.uint64(2)
    k = np.concatenate([pool_h[rng.integers(0, heavy_pool, n_heavy)], pool_l[rng.integers(0, light_pool, n_light)]])
    k = k[(k != root) & (k != np.uint64(2**64 - 1))]
    return k[rng.permutation(len(k))]


@pytest.mark.parametrize('order', [[0, 1, 2, 3], [3, 2, 1, 0], [2, 0, 3, 1]])
def test_claims_first_occurrence_under_contention(order):
    rng = np.random.default_rng(len(order) * 7 + order[0])
    keys = _keys(rng, 1_500_000, 3000, 1_500_000, 1_200_000)
    n = len(keys)
    first = np.zeros(n, np.uint8)
    _, idx = np.unique(keys, return_index=True)
    first[idx] = 1
    b = _backend(21)   # 2M slots for ~1.1M distinct keys: ~55% load, long probe chains
    try:
        dkeys = torch.from_numpy(keys.view(np.int64)).to(b.device)
        ret = b.answer_buffer(n)
        b.owner_begin(n, [0, 0])   # source 0 (this rank) sends nothing, source 1 all n records
        bounds = np.linspace(0, n, len(order) + 1).astype(np.int64)
        for c in order:   # chunks claimed out of index order: earlier records displace later holders
            a, e = int(bounds[c]), int(bounds[c + 1])
            b.owner_claim(dkeys[a:e], [0, 0], [0, a], ret)   # source 1's records a..e, answers at index a..
        b.owner_finish(ret)
        torch.cuda.synchronize()
        got = ret.cpu().numpy()
    finally:
        b.close()
    bad = np.nonzero(got != first)[0]
    assert len(bad) == 0, f'{len(bad)} records settled wrongly, first at {bad[:5]}'


def test_answer_bits_roundtrip():
    """sbd_pack_bits / sbd_unpack_bits (answers on the wire as bits) at unaligned offsets and lengths."""
    rng = np.random.default_rng(5)
    b = _backend(12)
    try:
        for n, off in ((0, 0), (1, 3), (7, 1), (8, 0), (9, 5), (1000, 13), (123457, 7)):
            src = (rng.random(n + off + 3) < 0.4).astype(np.uint8) * rng.integers(1, 255, n + off + 3).astype(np.uint8)
            ds = torch.from_numpy(src).to(b.device)
            packed = torch.zeros((n + 7) // 8 + 2, dtype=torch.uint8, device=b.device)
            b.pack_bits(ds[off:off + n], packed[1:1 + (n + 7) // 8])
            out = torch.full((n + off + 3,), 7, dtype=torch.uint8, device=b.device)
            b.unpack_bits(packed[1:1 + (n + 7) // 8], out[off:off + n])
            torch.cuda.synchronize()
            p = packed.cpu().numpy()
            want = np.packbits((src[off:off + n] != 0).astype(np.uint8), bitorder='little')
            assert np.array_equal(p[1:1 + len(want)], want) and p[0] == 0 and p[-1] == 0, n
            o = out.cpu().numpy()
            assert np.array_equal(o[off:off + n], (src[off:off + n] != 0).astype(np.uint8)), n
            assert (o[:off] == 7).all() and (o[off + n:] == 7).all(), n
    finally:
        b.close()


def test_answer_bits_segments_one_launch():
    """sbd_pack_bits_segs / sbd_unpack_bits_segs (every (source, part) answer segment in one launch) against
    numpy: 200 segments (more than one launch's table), empty and odd lengths, unaligned offsets, and bytes
    outside the segments left untouched."""
    rng = np.random.default_rng(11)
    b = _backend(12)
    try:
        lens = rng.integers(0, 3000, 200)
        lens[::17] = 0
        lens[5] = 1
        lens[6] = 8
        src_off = np.concatenate([[3], 3 + np.cumsum(lens + rng.integers(0, 5, 200))[:-1]]).astype(np.int64)
        nbytes = (lens + 7) // 8
        dst_off = np.concatenate([[1], 1 + np.cumsum(nbytes + 1)[:-1]]).astype(np.int64)
        src = (rng.random(int(src_off[-1] + lens[-1] + 8)) < 0.5).astype(np.uint8) * rng.integers(1, 255, int(src_off[-1] + lens[-1] + 8)).astype(np.uint8)
        ds = torch.from_numpy(src).to(b.device)
        packed = torch.zeros(int(dst_off[-1] + nbytes[-1] + 4), dtype=torch.uint8, device=b.device)
        segs = [(int(src_off[s]), int(lens[s]), int(dst_off[s])) for s in range(200)]
        b.pack_bits_segs(ds, segs, packed)
        out = torch.full_like(ds, 7)
        b.unpack_bits_segs(packed, [(int(dst_off[s]), int(lens[s]), int(src_off[s])) for s in range(200)], out)
        torch.cuda.synchronize()
        p, o = packed.cpu().numpy(), out.cpu().numpy()
        want_p = np.zeros_like(p)
        want_o = np.full_like(src, 7)
        for s in range(200):
            a, n, d = int(src_off[s]), int(lens[s]), int(dst_off[s])
            bits = np.packbits((src[a:a + n] != 0).astype(np.uint8), bitorder='little')
            want_p[d:d + len(bits)] = bits
            want_o[a:a + n] = (src[a:a + n] != 0).astype(np.uint8)
        assert np.array_equal(p, want_p)
        assert np.array_equal(o, want_o)
    finally:
        b.close()
