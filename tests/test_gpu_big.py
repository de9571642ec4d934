"""Parity at the benchmark configs' own widths (BASELINE.json configs[2..4]) against committed goldens of
the pinned C oracle (oracle/make_big_golden.py; the Python reference cannot run these widths here):

  * C4: realistic 2 players, goal 15, shuffled market seed 0, W=1M, one GPU
  * the sharded protocol at W=4M: world 1 (flags bit 1) on C3 (balanced; over gloo and over RCCL), and world 2 on one GPU (gloo
    transport, HIP per-rank primitives) on C5's heuristic (efficiency) — every turn's beam digest over the
    rank slices in rank order, turn sizes, path and final MT state
  * C5 itself (goal 15, efficiency, W=32M): the single-GPU engine (queues of >= 2^24 parents: 8-byte
    descriptors; the visited set rebuilt past 2^32 slots) and the sharded protocol at world 8 on one GPU
    (4M states per rank, gloo transport, HIP primitives: 8-way owner partition, 8-source claim segments)
"""
import json
import os
import random
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_c
from conftest import golden, golden_exists

pytestmark = pytest.mark.gpu


def test_realistic_c4_w1m_oracle_golden():
    from splendor_amd.engine_rt import RealisticEngine
    from splendor_amd.realistic import GameConfig, MultiPlayerState
    g = golden('oracle_realistic_g15_p2_shuf_w1000000_s0.json')
    cfg = GameConfig(num_players=2, target_points=15, gems_per_color=4, infinite_resources=False)
    root = MultiPlayerState.newgame(cfg, shuffle_market=True, seed=g['seed'])
    random.seed(g['seed'])
    eng = RealisticEngine(root, beam_width=g['beam_width'], mt_state625=random.getstate()[1])
    t = 0
    while True:
        s = eng.step()
        if s['done']:
            break
        t += 1
        exp = g['turns'][t - 1]
        assert (s['n_parents'], s['n_raw'], s['n_unique'], s['n_kept']) == \
            (exp['n_parents'], exp['n_raw'], exp['n_unique'], exp['n_kept']), t
        _, _, key = eng.read_turn(t)
        assert oracle_c.beam_digest(key) == exp['digest'], f'turn {t}'
    assert t == len(g['turns'])
    words = eng.path_words()
    assert [[f'{int(x):016x}' for x in row] for row in words] == g['path_words']
    assert oracle_c.mt_fingerprint(eng.mt_state()) == g['final_mt']
    eng.close()


def _wait_device_memory(min_free_gib=240.0, timeout_s=120.0, mem_get_info=None):
    """Wait until the device has released a previous multi-process test's memory (eight ranks of C5 need most
    of the 288 GB; the exited ranks' allocations are reclaimed asynchronously).  Fails the test (a precondition,
    not a protocol result) with the free and needed HBM when it does not come back in time."""
    import time
    if mem_get_info is None:
        import torch
        mem_get_info = lambda: torch.cuda.mem_get_info(0)
    t0 = time.time()
    free = 0
    while True:
        free, _ = mem_get_info()
        if free >= min_free_gib * 2**30:
            return free
        if time.time() - t0 >= timeout_s:
            break
        time.sleep(min(2.0, timeout_s / 4))
    pytest.fail(f'device memory not released in {timeout_s:.0f} s: {free / 2**30:.1f} GiB free, '
                f'{min_free_gib:.1f} GiB needed (a previous test\'s ranks still hold HBM; not a protocol failure)')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest_turn(outdir, t, world, order):
    """sha256 digest of turn t's beam over the rank slices in global order (runs (rank, start, length): block-cyclic
    slices interleave the ranks); the slices' files are removed."""
    fs = [os.path.join(outdir, f'keys_t{t}_r{r}.npy') for r in range(world)]
    ks = [np.load(f) for f in fs]
    key = np.concatenate([ks[r][a:a + n] for r, a, n in order])
    for f in fs:
        os.remove(f)
    return oracle_c.beam_digest(key), len(key)


def _worker(rank, world, port, cfg, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), 'splendor-rl-gym_amd'), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from splendor_amd.dist import Comm, DistSolve, HipBackend
    from splendor_amd.engine import HEURISTIC_IDS
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    backend = cfg.get('backend', 'gloo')
    if backend == 'nccl':   # RCCL: one rank per GPU (a world of one here), device bound at init as bench_dist does
        import torch
        torch.cuda.set_device(0)
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
    else:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    assert dist.get_backend() == backend
    random.seed(cfg['seed'])
    b = HipBackend(rank=rank, world=world, device_index=0, goal_pts=cfg['goal'], use_heuristic=True,
                   heuristic=HEURISTIC_IDS[cfg['heuristic']], beam_width=cfg['width'],
                   mt_state625=random.getstate()[1], visited_log2=cfg.get('visited_log2', 0),
                   extra_flags=cfg.get('flags', 0))
    if cfg.get('devdeferred'):   # Comm's RCCL branches under RCCL's device-side completion contract
        from device_deferred_comm import DeviceDeferredComm
        comm = DeviceDeferredComm(b.device)
    else:
        comm = Comm(b.device)
    solve = DistSolve(b, comm, goal_pts=cfg['goal'], use_heuristic=True, beam_width=cfg['width'])
    trace = []
    while True:
        st = solve.step()
        trace.append(st)
        if cfg.get('devdeferred'):
            comm.check_step()
        if st['done']:
            break
        np.save(os.path.join(outdir, f'keys_t{len(trace)}_r{rank}.npy'), b.turn_keys(len(trace)))
        if cfg.get('digest_inline'):   # wide beams: rank 0 digests each turn as it completes
            dist.barrier()
            if rank == 0:
                st['digest'], st['beam'] = _digest_turn(outdir, len(trace), world, solve.global_order(len(trace)))
                print(f'[world {world}] turn {len(trace)}: {st["n_parents"]} parents, digest {st["digest"]}',
                      flush=True)   # progress (pytest -s) for long runs
            dist.barrier()
    out = {'trace': trace, 'path': [list(x) for x in solve.path()], 'mt': b.mt_state().tolist(), 'bc': solve.bc,
           'order': [solve.global_order(t) for t in range(len(solve.blocks))],
           'visited_capacity': list(b.visited_capacity()),
           'deferred': [comm.deferred_calls, comm.waits, comm.landings] if cfg.get('devdeferred') else None}
    with open(os.path.join(outdir, f'rank{rank}.json'), 'w') as f:
        json.dump(out, f)
    b.close()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,name,backend,flags', [(1, 'oracle_g15_balanced_w4000000_s0.json', 'gloo', 0),
                                                      (1, 'oracle_g15_balanced_w4000000_s0.json', 'nccl', 0),
                                                      (2, 'oracle_g15_efficiency_w4000000_s0.json', 'gloo', 0),
                                                      (2, 'oracle_g15_efficiency_w4000000_s0.json', 'gloo', 256),
                                                      (2, 'oracle_g15_efficiency_w4000000_s0.json', 'devdeferred', 0),
                                                      (2, 'oracle_g15_efficiency_w4000000_s0.json', 'devdeferred', 768)])
def test_sharded_w4m_oracle_golden(world, name, backend, flags):
    """The sharded protocol at W=4M.  The nccl case is the C3 solve as `bench.py --gpus 1` with SB_FORCE_DIST=1
    runs it: init_process_group('nccl', device_id=...), the engine on torch's stream (sbd_set_stream) and
    Comm's RCCL branches (a world of one: RCCL refuses two ranks on one GPU).  The devdeferred cases run Comm's RCCL
    branches at world 2 under RCCL's device-side completion contract (tests/device_deferred_comm.py, gloo moving
    the data): the key-owner pipelined protocol and card-set ownership + owner emission (flags 768)."""
    g = golden(name)
    devdeferred = backend == 'devdeferred'
    cfg = {'goal': g['goal'], 'heuristic': g['heuristic'], 'width': g['beam_width'], 'seed': g['seed'],
           'backend': 'gloo' if devdeferred else backend, 'flags': flags,   # flags 256: card-set ownership (sb_mig.inc)
           'devdeferred': devdeferred}
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), cfg, d), nprocs=world, join=True)
        res = [json.load(open(os.path.join(d, f'rank{r}.json'))) for r in range(world)]
        turns = [t for t in res[0]['trace'] if not t['done']]
        assert len(turns) == len(g['turns'])
        for t, exp in enumerate(g['turns'], 1):
            a = turns[t - 1]
            assert (a['n_raw'], a['n_unique'], a['n_kept']) == (exp['n_raw'], exp['n_unique'], exp['n_kept']), t
            ks = [np.load(os.path.join(d, f'keys_t{t}_r{r}.npy')) for r in range(world)]
            key = np.concatenate([ks[r][a:a + n] for r, a, n in res[0]['order'][t]])
            assert oracle_c.beam_digest(key) == exp['digest'], f'turn {t}'
    from splendor_amd.codec import state_key, decode, to_signed
    path = [to_signed(state_key(decode(lo, hi)[0], decode(lo, hi)[2])) for lo, hi in res[0]['path']]
    assert path == [p[5] for p in g['path']]
    assert all(oracle_c.mt_fingerprint(r['mt']) == g['final_mt'] for r in res)
    if devdeferred:   # the async exchanges ran and each was waited for
        assert all(r['deferred'][0] > 0 and r['deferred'][0] == r['deferred'][1] for r in res), \
            [r['deferred'] for r in res]


C5 = 'oracle_g15_efficiency_w32000000_s0.json'


@pytest.mark.skipif(not golden_exists(C5), reason='C5 golden not generated')
def test_c5_w32m_single_gpu_oracle_golden():
    """C5's width on one MI355X: queues of 32M parents (>= 2^24: the top-k hands the gather 8-byte
    descriptors, sb_engine.hip desc_payload_ok) and a visited set started at 2^31 slots that is rebuilt
    (k_rehash) to 2^32 and then past it on the way to about 1.5G keys (flags bit 4: growth at 25%
    projected load, so a 2^32-slot table is itself rebuilt, 64-bit slot indices throughout)."""
    from splendor_amd import _lib as L
    from splendor_amd.engine import HEURISTIC_IDS, BeamEngine
    g = golden(C5)
    random.seed(g['seed'])
    eng = BeamEngine(goal_pts=g['goal'], use_heuristic=True, heuristic=HEURISTIC_IDS[g['heuristic']],
                     beam_width=g['beam_width'], mt_state625=random.getstate()[1], visited_log2=31, test_flags=16)
    t = 0
    while True:
        s = eng.step()
        if s['done']:
            break
        t += 1
        exp = g['turns'][t - 1]
        assert (s['n_parents'], s['n_raw'], s['n_unique'], s['n_kept']) == \
            (exp['n_parents'], exp['n_raw'], exp['n_unique'], exp['n_kept']), t
        _, _, _, key = eng.read_turn(t)
        assert oracle_c.beam_digest(key) == exp['digest'], f'turn {t}'
        del key
    assert t == len(g['turns'])
    from splendor_amd.codec import decode, state_key, to_signed
    assert [to_signed(state_key(decode(lo, hi)[0], decode(lo, hi)[2])) for lo, hi in eng.path()] == \
        [p[5] for p in g['path']]
    assert oracle_c.mt_fingerprint(eng.mt_state()) == g['final_mt']
    cap, rebuilds = L.visited_capacity(eng._h)
    assert eng.visited_size() == g['visited']
    assert cap > (1 << 32) and rebuilds >= 2, (cap, rebuilds)
    eng.close()


@pytest.mark.skipif(not golden_exists(C5), reason='C5 golden not generated')
@pytest.mark.parametrize('mig', [False, True, 'oe'])
def test_c5_sharded_world8_oracle_golden(mig):
    """C5 as the 8-GPU job runs it, 8 ranks on one GPU (gloo transport, HIP per-rank primitives, 4M
    states per rank): every turn's digest over the rank slices, sizes, path, final MT state on every
    rank; each rank's owner shard starts at 2^28 slots and is rebuilt on the way; record buffers sized for
    48 raw children per parent, flags bit 5, since eight ranks share one GPU's HBM)."""
    g = golden(C5)
    world = 8
    cfg = {'goal': g['goal'], 'heuristic': g['heuristic'], 'width': g['beam_width'], 'seed': g['seed'],
           'visited_log2': 28, 'digest_inline': True,
           'flags': 32 | (256 if mig else 0) | (512 if mig == 'oe' else 0)}   # 8 ranks share one GPU's HBM; 256:
    # card-set ownership; 512: owner emission
    _wait_device_memory()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), cfg, d), nprocs=world, join=True)
        res = [json.load(open(os.path.join(d, f'rank{r}.json'))) for r in range(world)]
    turns = [t for t in res[0]['trace'] if not t['done']]
    assert len(turns) == len(g['turns'])
    for t, exp in enumerate(g['turns'], 1):
        a = turns[t - 1]
        assert (a['n_raw'], a['n_unique'], a['n_kept']) == (exp['n_raw'], exp['n_unique'], exp['n_kept']), t
        assert (a['digest'], a['beam']) == (exp['digest'], exp['n_kept']), f'turn {t}'
    from splendor_amd.codec import decode, state_key, to_signed
    path = [to_signed(state_key(decode(lo, hi)[0], decode(lo, hi)[2])) for lo, hi in res[0]['path']]
    assert path == [p[5] for p in g['path']]
    assert all(oracle_c.mt_fingerprint(r['mt']) == g['final_mt'] for r in res)
    assert all(r['visited_capacity'][1] >= 1 for r in res)
