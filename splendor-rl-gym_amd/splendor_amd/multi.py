"""Multi-GPU solve from the drop-in surface: ``State.solve(gpus=N)`` and the CLI's ``--gpus N``.

The reference has one entry point for a solve (``State.solve``, src/solver.py:390-464, called by
splendor_fastest_win.py:130-145).  With ``gpus > 1`` the calling process starts one worker per GPU with
``torch.distributed.run`` (a child process: the caller never initialises the GPU for this), the workers
run the sharded step (``dist.DistSolve`` over ``HipBackend``; RCCL, or gloo with
``SB_DIST_BACKEND=gloo``), rank 0 prints exactly the lines the single-GPU solve prints (``turn=`` /
``max_pts=``) and hands the path and the final MT19937 state back through a file; the caller returns
``State`` objects and leaves ``random`` where the reference would.  Results are bit-identical to one
GPU (the sharded protocol's parity tests).

    python -m torch.distributed.run --nproc-per-node N -m splendor_amd.multi SPEC.json OUT.json
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import tempfile

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(spec: dict, gpus: int) -> dict:
    """Run the sharded solve described by `spec` on `gpus` worker processes; returns rank 0's result
    (``{'path': [[lo, hi], ...], 'mt': [625 ints]}``, or the world size for a dry run)."""
    if gpus < 1:
        raise ValueError('gpus must be >= 1')
    with tempfile.TemporaryDirectory(prefix='sb_multi_') as d:
        sp, op = os.path.join(d, 'spec.json'), os.path.join(d, 'out.json')
        with open(sp, 'w') as f:
            json.dump(spec, f)
        env = dict(os.environ)
        env['PYTHONPATH'] = PKG_ROOT + (os.pathsep + env['PYTHONPATH'] if env.get('PYTHONPATH') else '')
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={gpus}',
               '--master-addr=127.0.0.1', f'--master-port={_free_port()}', '-m', 'splendor_amd.multi', sp, op]
        sys.stdout.flush()
        rc = subprocess.call(cmd, env=env)
        if rc != 0 or not os.path.exists(op):
            raise RuntimeError(f'sharded solve on {gpus} GPUs failed (launcher exit code {rc})')
        with open(op) as f:
            return json.load(f)


def _state_at(solve, t: int, r: int):
    """(lo, hi) of global queue position r of turn t; a collective (every rank calls it)."""
    owner, loc = solve.locate(t, r)   # (block-cyclic slices interleave the ranks)
    vals = [0, 0, 0]
    if owner == solve.c.rank:
        from .dist import _u64_to_i64
        lo, hi, par = solve.b.turn_state(t, loc)
        vals = [_u64_to_i64(lo), _u64_to_i64(hi), par]
    lo, hi, _ = solve.c.broadcast_ints(vals, owner)
    return lo & 0xFFFFFFFFFFFFFFFF, hi & 0xFFFFFFFFFFFFFFFF


def worker(spec_path: str, out_path: str) -> None:
    # RCCL prints a banner on stdout at init: stdout is kept for rank 0's solve lines only
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    with open(spec_path) as f:
        spec = json.load(f)
    world = int(os.environ['WORLD_SIZE'])
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if spec.get('dry_run'):
        dist.init_process_group('gloo')
        dist.barrier()
        if dist.get_rank() == 0:
            with open(out_path, 'w') as f:
                json.dump({'dry_run': True, 'world': dist.get_world_size()}, f)
        dist.destroy_process_group()
        return
    backend = os.environ.get('SB_DIST_BACKEND', 'nccl')
    ndev = torch.cuda.device_count()
    dev = spec.get('device', 0) + local if backend == 'nccl' else (spec.get('device', 0) + local) % max(ndev, 1)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, device_id=torch.device('cuda', dev) if backend == 'nccl' else None)
    from .dist import Comm, DistSolve, HipBackend
    from .solver import State
    rank = dist.get_rank()
    assert dist.get_world_size() == world
    b = HipBackend(rank=rank, world=world, device_index=dev, goal_pts=spec['goal'],
                   use_heuristic=spec['use_heuristic'], heuristic=spec['heuristic'], beam_width=spec['beam_width'],
                   mt_state625=spec['mt'], root=tuple(spec['root']))
    solve = DistSolve(b, Comm(b.device), goal_pts=spec['goal'], use_heuristic=spec['use_heuristic'],
                      beam_width=spec['beam_width'])
    out = os.fdopen(out_fd, 'w') if rank == 0 else None
    verbose = spec['verbose']
    turn = 0
    while True:
        if verbose:
            s = State.from_packed(*_state_at(solve, turn, 0))
            if out:
                print(f'turn={turn:<10} {s}', file=out, flush=True)
        st = solve.step()
        if verbose:
            for r, pts in st['records']:
                s = State.from_packed(*_state_at(solve, turn, r))
                if out:
                    print(f'max_pts={pts:<7} {s}', file=out, flush=True)
        if st['done']:
            break
        turn += 1
    path = solve.path()
    mt = b.mt_state().tolist()
    if rank == 0:
        with open(out_path, 'w') as f:
            json.dump({'path': [[int(lo), int(hi)] for lo, hi in path], 'mt': [int(x) for x in mt],
                       'world': world}, f)
        out.close()
    b.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    worker(sys.argv[1], sys.argv[2])
