"""Sharded multi-rank protocol (splendor_amd.dist) on CPU with gloo, world sizes 2, 3, 4 and 8.

Every rank runs DistSolve over the Python reference backend; the concatenated rank slices of every
turn must equal the single-process oracle's queue (keys, parent links), and the path and final MT
state must match.  This is the N>1 path of bench.py with the per-rank compute swapped for the
reference primitives.
"""
import json
import os
import random
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_c


def _worker(rank, world, port, cfg, outdir):
    if 'gkr' in cfg:   # grouped kept records on the rebalance's wire (dist.GKR, read at import)
        os.environ['SB_DIST_GKR'] = '1' if cfg['gkr'] else '0'
    if 'p0' in cfg:   # block-cyclic: part 0's blocks relative to the others' (dist.P0, read at import)
        os.environ['SB_DIST_P0'] = str(cfg['p0'])
    if 'chunks' in cfg:
        os.environ['SB_DIST_CHUNKS'] = str(cfg['chunks'])
        os.environ['SB_DIST_CHUNK_MIN'] = '0'
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), 'splendor-rl-gym_amd'),
              os.path.join(os.path.dirname(here), 'oracle'), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from dist_ref_backend import RefBackend
    from splendor_amd.dist import Comm, DistSolve
    # a file store in the test's directory: no TCP port to pick and lose to a parallel test worker before binding
    dist.init_process_group('gloo', init_method='file://' + os.path.join(outdir, 'store'), rank=rank, world_size=world)
    random.seed(cfg['seed'])
    st = random.getstate()[1]
    b = RefBackend(rank, heuristic=cfg['hid'], mt_state625=st, world=world)
    b.parts = cfg.get('parts', 0)   # > 0: the pipelined protocol (the HIP key pass's exchange parts)
    if cfg.get('mig'):   # card-set ownership of the trail (sb_mig.inc restated); 'force0': every card set to rank 0
        b.mig, b.force0 = True, cfg.get('force0', False)
        b.oe = cfg.get('oe', False)   # owner emission: survivors emitted on the expanding ranks
        b.parts = b.parts or 2
    if cfg.get('goc'):   # global-order claims (HipBackend.GOC): own children as records, one claim pass
        b.goc = True
    if cfg.get('small_cap'):   # a receive bound far below the records received: the host grows it (sbd_grow_receive)
        b.recv_cap = cfg['small_cap']
    if cfg.get('shm'):   # every rank on this node (torch.distributed.run sets it): host metadata over shared memory
        os.environ['LOCAL_WORLD_SIZE'] = str(world)
    if cfg.get('deferred'):   # RCCL's completion contract (Comm's non-gloo branches), tests/deferred_comm.py
        from deferred_comm import DeferredComm
        comm = DeferredComm(torch.device('cpu'))
    else:
        comm = Comm(torch.device('cpu'))
    if cfg.get('shm'):
        assert comm.shm is not None, 'shared-memory metadata not set up'
    if cfg.get('serialize'):   # the profiling wrappers (bench_dist.py SB_DIST_SERIALIZE=1) change nothing
        from splendor_amd.dist import SerializedBackend
        b = SerializedBackend(b)
        comm.devlock = b.lock
    solve = DistSolve(b, comm, goal_pts=cfg['goal'], use_heuristic=cfg['heur'],
                      beam_width=cfg['width'])
    trace = []
    while not solve.done:
        if cfg.get('toggle'):   # bench.py's window edges: the next turn's expansion deferred to the next step
            solve.lookahead = len(trace) % 3 != 1
        trace.append(solve.step())
        if cfg.get('deferred'):
            assert not comm.outstanding, f'step {len(trace)} left an all_to_all handle unwaited'
    out = {'trace': trace, 'counts': [c.tolist() for c in solve.counts], 'path': [list(x) for x in solve.path()],
           'order': [solve.global_order(t) for t in range(len(solve.blocks))], 'bc': solve.bc,
           'slices': [[lo, hi, par] for lo, hi, par in b.turns],
           'mt': b.mt_state().tolist() if cfg['heur'] else None,
           'deferred': [comm.deferred_calls, comm.waits] if cfg.get('deferred') else None,
           'grown': getattr(b, 'grown', 0), 'shm': getattr(comm, 'shm', None) is not None,
           'collectives': [t.get('collectives') for t in trace]}
    with open(os.path.join(outdir, f'rank{rank}.json'), 'w') as f:
        json.dump(out, f)
    dist.destroy_process_group()


def _run(world, cfg):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, None, cfg, d), nprocs=world, join=True)
        return [json.load(open(os.path.join(d, f'rank{r}.json'))) for r in range(world)]


def assemble(res, t, i):
    """Field i of turn t's queue in global order from the rank slices (block-cyclic slices: blocks j-major)."""
    return sum((res[r]['slices'][t][i][a:a + n] for r, a, n in res[0]['order'][t]), [])


CASES = [
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True}),
    (3, {'goal': 5, 'hid': 0, 'name': 'simple', 'width': 97, 'seed': 2, 'heur': True}),
    (2, {'goal': 7, 'hid': 3, 'name': 'efficiency', 'width': 40, 'seed': 3, 'heur': True}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False}),
    # key exchange in 3 chunks (claims in chunk order, displacements across chunks)
    (2, {'goal': 6, 'hid': 2, 'name': 'aggressive', 'width': 600, 'seed': 5, 'heur': True, 'chunks': 3}),
    # the driver's scaling runs use 4 and 8 ranks
    (4, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 250, 'seed': 7, 'heur': True, 'chunks': 2}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True}),
    # lookahead off every third step (the expansion launched by the step that needs it)
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 9, 'heur': True, 'toggle': True}),
    # the per-rank profiling wrapper (one rank's backend calls at a time) changes no result
    (3, {'goal': 5, 'hid': 1, 'name': 'balanced', 'width': 200, 'seed': 4, 'heur': True, 'serialize': True}),
    # the pipelined protocol: records exchanged and claimed part by part, answer-index tags
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'parts': 3}),
    (3, {'goal': 5, 'hid': 0, 'name': 'simple', 'width': 97, 'seed': 2, 'heur': True, 'parts': 2}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'parts': 2}),
    (4, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 250, 'seed': 7, 'heur': True, 'parts': 1}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True, 'parts': 4}),
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 9, 'heur': True, 'toggle': True, 'parts': 4}),
    (3, {'goal': 5, 'hid': 1, 'name': 'balanced', 'width': 200, 'seed': 4, 'heur': True, 'serialize': True,
         'parts': 2}),
    # the 20-byte kept records instead of (parent, destination) groups on the rebalance's wire
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'parts': 3, 'gkr': False}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True, 'parts': 4, 'gkr': False}),
    # Comm's RCCL branches under RCCL's completion contract (deferred receive buffers, poisoned until
    # wait): the pipelined protocol at worlds 2/4/8 and the chunked legacy exchange
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'parts': 3, 'deferred': True}),
    (4, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 250, 'seed': 7, 'heur': True, 'parts': 4, 'deferred': True}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True, 'parts': 2,
         'deferred': True}),
    (4, {'goal': 6, 'hid': 2, 'name': 'aggressive', 'width': 600, 'seed': 5, 'heur': True, 'chunks': 3,
         'deferred': True}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'parts': 2, 'deferred': True}),
    # card-set ownership: parents migrate to their card-set owners, takes claimed there, buys exchanged as
    # (key, tag) records; the survivor masks come back to the slice's rank
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'mig': True}),
    (3, {'goal': 5, 'hid': 0, 'name': 'simple', 'width': 97, 'seed': 2, 'heur': True, 'mig': True, 'parts': 3}),
    (4, {'goal': 6, 'hid': 2, 'name': 'aggressive', 'width': 600, 'seed': 5, 'heur': True, 'mig': True,
         'deferred': True}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True, 'mig': True, 'parts': 1}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'mig': True}),
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 9, 'heur': True, 'toggle': True, 'mig': True}),
    (3, {'goal': 5, 'hid': 1, 'name': 'balanced', 'width': 200, 'seed': 4, 'heur': True, 'mig': True, 'force0': True}),
    # owner emission: the survivors emitted on the expanding ranks (offsets and noise draws sent there), ties at the
    # keep boundary by next_queue position over all ranks, the receiver orders by (score, position)
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'mig': True, 'oe': True}),
    (3, {'goal': 5, 'hid': 0, 'name': 'simple', 'width': 97, 'seed': 2, 'heur': True, 'mig': True, 'oe': True,
         'parts': 3}),
    (4, {'goal': 6, 'hid': 2, 'name': 'aggressive', 'width': 600, 'seed': 5, 'heur': True, 'mig': True, 'oe': True,
         'deferred': True}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True, 'mig': True, 'oe': True,
         'parts': 1}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'mig': True, 'oe': True}),
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 9, 'heur': True, 'toggle': True, 'mig': True,
         'oe': True}),
    (3, {'goal': 5, 'hid': 1, 'name': 'balanced', 'width': 200, 'seed': 4, 'heur': True, 'mig': True, 'force0': True,
         'oe': True}),
    # the receive bound (an estimate) exceeded mid-turn: grown from the exact counts instead of failing
    (3, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'parts': 3, 'small_cap': 8}),
    (2, {'goal': 6, 'hid': 2, 'name': 'aggressive', 'width': 600, 'seed': 5, 'heur': True, 'parts': 2, 'small_cap': 8,
         'deferred': True}),
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'mig': True, 'small_cap': 8}),
    # global-order claims: the own children become records to this rank, every record of the turn is claimed in one
    # pass in (source, part, record) order once all parts arrived; answers by virtual index
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'parts': 3, 'goc': True}),
    (3, {'goal': 5, 'hid': 0, 'name': 'simple', 'width': 97, 'seed': 2, 'heur': True, 'parts': 2, 'goc': True}),
    (4, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 250, 'seed': 7, 'heur': True, 'parts': 4, 'goc': True,
         'deferred': True}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True, 'parts': 2, 'goc': True,
         'deferred': True}),
    (2, {'goal': 3, 'hid': 0, 'name': 'simple', 'width': 1, 'seed': 0, 'heur': False, 'parts': 2, 'goc': True}),
    (3, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'parts': 3, 'goc': True,
         'small_cap': 8, 'deferred': True}),
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 9, 'heur': True, 'toggle': True, 'parts': 4,
         'goc': True}),
    # block-cyclic slices (the default with global-order claims): 16 blocks per rank at world 3 and 4 (48 / 64
    # boundaries: 8-bit select digits), one rank (the KP1 measurement's world-1 protocol), 20-byte records refuse them
    (3, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 400, 'seed': 13, 'heur': True, 'parts': 16, 'goc': True}),
    (4, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 500, 'seed': 14, 'heur': True, 'parts': 16, 'goc': True,
         'deferred': True}),
    (1, {'goal': 6, 'hid': 2, 'name': 'aggressive', 'width': 300, 'seed': 15, 'heur': True, 'parts': 4, 'goc': True}),
    (2, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 300, 'seed': 1, 'heur': True, 'parts': 3, 'goc': True,
         'gkr': False}),
    # host metadata over shared memory (ShmMeta: the default when every rank is on one node)
    (4, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 250, 'seed': 7, 'heur': True, 'parts': 4, 'goc': True,
         'shm': True}),
    (8, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 120, 'seed': 8, 'heur': True, 'parts': 2, 'goc': True,
         'shm': True}),
    # part 0's blocks a third / twice the others' (SB_DIST_P0): any boundaries, the same on every rank
    (3, {'goal': 6, 'hid': 1, 'name': 'balanced', 'width': 400, 'seed': 13, 'heur': True, 'parts': 4, 'goc': True,
         'p0': 0.33}),
    (2, {'goal': 5, 'hid': 3, 'name': 'efficiency', 'width': 300, 'seed': 14, 'heur': True, 'parts': 3, 'goc': True,
         'p0': 2.0, 'deferred': True}),
]


@pytest.mark.parametrize('world,cfg', CASES)
def test_sharded_solve_matches_oracle(world, cfg):
    res = _run(world, cfg)
    random.seed(cfg['seed'])
    st = random.getstate()[1]
    o = oracle_c.OracleSolve(cfg['goal'], use_heuristic=cfg['heur'], heuristic_name=cfg['name'],
                             beam_width=cfg['width'], mt_state625=st)
    trace = o.run()
    assert [t['done'] for t in res[0]['trace']] == [t['done'] for t in trace]
    for t in range(o.nturns()):
        lo, hi, par, _ = o.turn_arrays(t)
        glo, ghi, gpar = (assemble(res, t, i) for i in range(3))
        assert glo == lo.tolist() and ghi == hi.tolist(), f'turn {t}'
        if t > 0:
            assert gpar == par.tolist(), f'turn {t} parents'
    for a, b in zip(res[0]['trace'], trace):
        assert a['n_parents'] == b['n_parents'] and a['records'] == [tuple(x) for x in b['records']] or \
            [list(x) for x in a['records']] == [list(x) for x in b['records']]
        if not b['done']:
            assert (a['n_raw'], a['n_unique'], a['n_kept']) == (b['n_raw'], b['n_unique'], b['n_kept'])
    path = [tuple(p) for p in res[0]['path']]
    assert path == o.path()
    assert all([tuple(p) for p in r['path']] == path for r in res)
    if cfg['heur']:
        assert all(r['mt'] == o.mt_state().tolist() for r in res)
    if cfg.get('small_cap'):
        assert any(r['grown'] for r in res), 'no rank grew its receive bound'
    if cfg.get('goc') and cfg['heur'] and cfg.get('parts', 0) >= 2:   # block-cyclic unless 20-byte records
        assert res[0]['bc'] == (cfg.get('gkr', True) or world == 1), res[0]['bc']
    if cfg.get('shm'):   # the metadata went over shared memory: one host round per turn sync and per part
        assert all(r['shm'] for r in res)
        P = cfg['parts']
        assert all(c is None or c[1] == 1 + P for r in res for c in r['collectives'][1:-1]), res[0]['collectives']
    if cfg.get('deferred'):   # the deferred path really ran: every rank issued async exchanges and waited for each
        assert all(r['deferred'][0] > 0 and r['deferred'][0] == r['deferred'][1] for r in res), [r['deferred'] for r in res]
    o.close()


def _shm_worker(rank, world, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), 'splendor-rl-gym_amd')):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from splendor_amd.dist import ShmMeta
    dist.init_process_group('gloo', init_method='file://' + os.path.join(outdir, 'store'), rank=rank, world_size=world)
    g = dist.new_group(backend='gloo')
    m = ShmMeta(rank, world, g)
    rng = np.random.default_rng(100 + rank)
    for k in range(200):   # rounds of varying lengths (both parity slots reused many times), ranks skewed
        n = 1 + (k * 37) % ShmMeta.SLOT
        v = np.arange(n, dtype=np.int64) * (rank + 1) + k
        if rng.random() < 0.1:
            import time
            time.sleep(0.002)
        out = m.allgather(v)
        exp = np.stack([np.arange(n, dtype=np.int64) * (q + 1) + k for q in range(world)])
        assert out.shape == (world, n) and (out == exp).all(), (rank, k)
    m.close()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 5])
def test_shm_meta_allgather(world):
    """ShmMeta (the host metadata exchange when every rank is on one node): 200 all_gathers of varying length with
    skewed ranks return every rank's vector in rank order."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_shm_worker, args=(world, d), nprocs=world, join=True)
