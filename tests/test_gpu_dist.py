"""Sharded engine on the GPU: world 2/3 ranks on one MI355X (gloo transport, HIP per-rank primitives).

Each rank runs DistSolve over HipBackend (sbd_* entry points of libsplendor_beam.so); the rank slices
of every turn, concatenated, must equal the oracle's queue (keys and parent links), and the path and
MT state must match.  (RCCL needs one GPU per rank; the 8-GPU RCCL run is bench.py --gpus N.)
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

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, outdir):
    if 'chunks' in cfg:
        os.environ['SB_DIST_CHUNKS'] = str(cfg['chunks'])
        os.environ['SB_DIST_CHUNK_MIN'] = '0'
    if 'ck' in cfg:
        os.environ['SB_NOISE_CK'] = str(cfg['ck'])
    if 'keypass' in cfg:   # 0: the expansion kernel + separate owner partition (sbd_expand_launch) at world > 1
        os.environ['SB_DIST_KEYPASS'] = str(cfg['keypass'])
    if cfg.get('kp1'):     # the world > 1 key-owner path at world 1 (HipBackend.KP1, a measurement aid)
        os.environ['SB_DIST_KP1'] = '1'
    if 'gkr' in cfg:       # grouped kept records on the rebalance's wire (default on)
        os.environ['SB_DIST_GKR'] = '1' if cfg['gkr'] else '0'
    if 'parts' in cfg:     # exchange parts of the pipelined key pass (default 4)
        os.environ['SB_DIST_PARTS'] = str(cfg['parts'])
    if cfg.get('nobc'):    # contiguous rank ranges instead of block-cyclic slices
        os.environ['SB_DIST_BC'] = '0'
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), 'splendor-rl-gym_amd'),
              os.path.join(os.path.dirname(here), 'oracle'), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from splendor_amd.dist import Comm, DistSolve, HipBackend
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    random.seed(cfg['seed'])
    st = random.getstate()[1]
    b = HipBackend(rank=rank, world=world, device_index=0, goal_pts=cfg['goal'], use_heuristic=cfg['heur'],
                   heuristic=cfg['hid'], beam_width=cfg['width'], mt_state625=st, visited_log2=cfg.get('vlog2', 0),
                   extra_flags=cfg.get('flags', 0))
    if cfg.get('shm'):   # every rank on this node, as under torch.distributed.run: metadata over shared memory
        os.environ['LOCAL_WORLD_SIZE'] = str(world)
    if cfg.get('devdeferred'):   # Comm's RCCL branches under RCCL's device-side completion contract
        from device_deferred_comm import DeviceDeferredComm
        comm = DeviceDeferredComm(b.device)
    else:
        comm = Comm(b.device)
    if cfg.get('shm'):
        assert comm.shm is not None
    solve = DistSolve(b, comm, goal_pts=cfg['goal'], use_heuristic=cfg['heur'], beam_width=cfg['width'])
    trace = []
    while not solve.done:
        trace.append(solve.step())
        if cfg.get('devdeferred'):
            comm.check_step()
    slices = []
    for t in range(len(solve.counts)):
        n = int(solve.counts[t][rank])
        rows = [b.turn_state(t, r) for r in range(n)]
        slices.append([[x[0] for x in rows], [x[1] for x in rows], [x[2] for x in rows]])
    out = {'trace': trace, 'path': [list(x) for x in solve.path()], 'slices': slices, 'bc': solve.bc,
           'order': [solve.global_order(t) for t in range(len(solve.blocks))],
           'mt': b.mt_state().tolist(), 'visited': list(b.visited_capacity()),
           'deferred': [comm.deferred_calls, comm.waits, comm.landings] if cfg.get('devdeferred') else None}
    with open(os.path.join(outdir, f'rank{rank}.json'), 'w') as f:
        json.dump(out, f)
    b.close()
    dist.destroy_process_group()


CASES = [
    (2, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 700, 'seed': 1, 'heur': True}),
    (3, {'goal': 6, 'hid': 0, 'name': 'simple', 'width': 250, 'seed': 2, 'heur': True}),
    (2, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False}),
    # 8 twists per producer segment, a checkpoint window every twist: sub-segment windows cross ranks
    (2, {'goal': 8, 'hid': 2, 'name': 'aggressive', 'width': 40000, 'seed': 4, 'heur': True, 'ck': 1}),
    # key exchange in 3 chunks (claims in chunk order, displacements across chunks)
    (3, {'goal': 7, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 6, 'heur': True, 'chunks': 3}),
    # four ranks on the one GPU (the driver's scaling runs use 2, 4 and 8 GPUs)
    (4, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 9, 'heur': True, 'chunks': 2}),
    # owner shards from a 1024-slot table: rebuilt larger between turns (unbounded trail)
    (2, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 5000, 'seed': 10, 'heur': True, 'vlog2': 10}),
    # the legacy expansion (k_expand<true> + stable owner partition) beside the default key pass
    (2, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 700, 'seed': 1, 'heur': True, 'keypass': 0}),
    (3, {'goal': 7, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 6, 'heur': True, 'chunks': 3, 'keypass': 0}),
    # the pipelined key pass in one part, and in 16 (parts of a few chunks, some empty on small turns)
    (2, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'parts': 1}),
    (3, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 11, 'heur': True, 'parts': 16}),
    # every key owned by rank 0 (flags bit 7): rank 0's parts send no records, so the apply must see its own
    # children marked (k_keys_b runs without a send buffer), never a previous turn's record positions
    (2, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'flags': 128}),
    (3, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 5000, 'seed': 12, 'heur': True, 'flags': 128, 'parts': 3}),
    # card-set ownership of the trail (flags bit 8, sb_mig.inc): parents migrate to their card-set owners,
    # takes are claimed where generated, buys exchanged as (key, tag) records, masks back to the slice's rank
    (2, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 700, 'seed': 1, 'heur': True, 'flags': 256}),
    (3, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'flags': 256}),
    (4, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 9, 'heur': True, 'flags': 256}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'flags': 256}),
    (2, {'goal': 8, 'hid': 2, 'name': 'aggressive', 'width': 40000, 'seed': 4, 'heur': True, 'ck': 1, 'flags': 256,
         'parts': 1}),
    (3, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 11, 'heur': True, 'flags': 256, 'parts': 16}),
    (2, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 5000, 'seed': 10, 'heur': True, 'vlog2': 10, 'flags': 256}),
    # every card set owned by rank 0: the other ranks expand nothing, rank 0 sends no records
    (3, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 5000, 'seed': 12, 'heur': True, 'flags': 384}),
    # owner emission (flags bit 9, sb_oe.inc): survivors emitted on the expanding ranks with the offsets and draws
    # the range ranks send; keep-boundary ties by position over all ranks; receivers order by (score, position)
    (2, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 700, 'seed': 1, 'heur': True, 'flags': 768}),
    (3, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'flags': 768}),
    (4, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 9, 'heur': True, 'flags': 768}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'flags': 768}),
    (2, {'goal': 8, 'hid': 2, 'name': 'aggressive', 'width': 40000, 'seed': 4, 'heur': True, 'ck': 1, 'flags': 768,
         'parts': 1}),
    (3, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 5000, 'seed': 12, 'heur': True, 'flags': 896}),
    # the receive bound starts at 1024 records (flags bit 10): every turn past it grows the lost bits / tags and the
    # answer buffer from the exact counts, mid-turn, with earlier parts' claims kept (sbd_grow_receive)
    (3, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 11, 'heur': True, 'flags': 1024, 'parts': 4}),
    (2, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'flags': 1024 | 256}),
    # the key-owner path (pipelined key pass, global-order claims of the own children as records) at world 1: the
    # one-GPU measurement of a rank's sharded device work (bench.py SB_FORCE_DIST=1 SB_DIST_KP1=1)
    (1, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'kp1': True}),
    (1, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 9, 'heur': True, 'kp1': True, 'parts': 3}),
    # kept records on the rebalance's wire: the 20-byte records instead of (parent, destination) groups
    (3, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 11, 'heur': True, 'gkr': False}),
    # Comm's RCCL branches against the engine's two streams, under RCCL's device-side completion contract
    # (tests/device_deferred_comm.py: receive buffers poisoned and filled late on a side stream, consumers ordered
    # only by the waits the protocol makes, send pieces checked unchanged until completion): key ownership
    # pipelined in 4 parts, card-set ownership + owner emission, the legacy chunked exchange, pure BFS
    (2, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 700, 'seed': 1, 'heur': True, 'devdeferred': True}),
    (4, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 9, 'heur': True, 'devdeferred': True}),
    (4, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'flags': 768,
         'devdeferred': True}),
    (2, {'goal': 8, 'hid': 2, 'name': 'aggressive', 'width': 40000, 'seed': 4, 'heur': True, 'flags': 768,
         'devdeferred': True}),
    (3, {'goal': 7, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 6, 'heur': True, 'chunks': 3, 'keypass': 0,
         'devdeferred': True}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'devdeferred': True}),
    # block-cyclic slices (the default of the key-owner protocol): each exchange part one block of the global queue,
    # claimed as soon as it has arrived; 16 blocks per rank at world 3 (48 boundaries: 8-bit select digits), the RCCL
    # contract at world 4, one rank in 4 blocks (the KP1 measurement), and the contiguous slices it replaces
    (3, {'goal': 8, 'hid': 1, 'name': 'balanced', 'width': 20000, 'seed': 11, 'heur': True, 'parts': 16, 'bc': True}),
    (4, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'devdeferred': True,
         'bc': True}),
    (1, {'goal': 8, 'hid': 2, 'name': 'aggressive', 'width': 40000, 'seed': 4, 'heur': True, 'kp1': True, 'ck': 1,
         'bc': True}),
    (2, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 5000, 'seed': 10, 'heur': True, 'vlog2': 10, 'bc': True}),
    (2, {'goal': 7, 'hid': 1, 'name': 'balanced', 'width': 700, 'seed': 1, 'heur': True, 'nobc': True, 'bc': False}),
    (4, {'goal': 8, 'hid': 3, 'name': 'efficiency', 'width': 3000, 'seed': 3, 'heur': True, 'shm': True, 'bc': True}),
]


@pytest.mark.parametrize('world,cfg', CASES)
def test_sharded_engine_matches_oracle(world, cfg):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), cfg, d), nprocs=world, join=True)
        res = [json.load(open(os.path.join(d, f'rank{r}.json'))) for r in range(world)]
    random.seed(cfg['seed'])
    st = random.getstate()[1]
    o = oracle_c.OracleSolve(cfg['goal'], use_heuristic=cfg['heur'], heuristic_name=cfg['name'],
                             beam_width=cfg['width'], mt_state625=st)
    trace = o.run()
    assert len(res[0]['trace']) == len(trace)
    asm = lambda t, i: sum((res[r]['slices'][t][i][a:a + n] for r, a, n in res[0]['order'][t]), [])   # global order
    for t in range(o.nturns()):
        lo, hi, par, _ = o.turn_arrays(t)
        assert asm(t, 0) == lo.tolist(), f'turn {t}'
        assert asm(t, 1) == hi.tolist(), f'turn {t}'
        if t > 0:
            assert asm(t, 2) == par.tolist(), f'turn {t} parents'
    if cfg.get('bc') is not None:
        assert res[0]['bc'] == cfg['bc'], res[0]['bc']
    for a, b in zip(res[0]['trace'], trace):
        if not b['done']:
            assert (a['n_raw'], a['n_unique'], a['n_kept']) == (b['n_raw'], b['n_unique'], b['n_kept'])
    assert [tuple(p) for p in res[0]['path']] == o.path()
    if cfg['heur']:
        assert all(r['mt'] == o.mt_state().tolist() for r in res)
    if cfg.get('devdeferred'):   # the RCCL branches really ran: async exchanges issued and each waited for
        assert all(r['deferred'][2] > 0 for r in res), [r['deferred'] for r in res]
        if world > 1 and cfg.get('keypass', 1):
            assert all(r['deferred'][0] > 0 and r['deferred'][0] == r['deferred'][1] for r in res), \
                [r['deferred'] for r in res]
    if 'vlog2' in cfg:
        assert all(r['visited'][1] >= 2 and r['visited'][0] > (1 << cfg['vlog2']) for r in res), res[0]['visited']
    o.close()
