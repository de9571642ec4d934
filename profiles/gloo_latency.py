#!/usr/bin/env python3
"""Host collective latency of the sharded step's metadata exchanges, measured on CPU alone.

The key-owner step's host round trips go over a gloo group (Comm.meta, splendor_amd/dist.py): the turn sync (one
all_gather of 257 + parts int64 per rank) and, per exchange part, the part's per-owner record counts (world + 1 int64).
Eight processes on one host, as an 8-GPU node runs them, time each kind of all_gather (median and p90 over many
rounds, after a warmup) over gloo and over shared memory (ShmMeta, the default since round 6) — no GPU involved.
    python3 profiles/gloo_latency.py [--world 8] [--rounds 400] [--out profiles/r6/gloo_latency.json]
"""
import argparse
import json
import os
import socket
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, rounds, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    meta = dist.new_group(backend='gloo')   # as Comm.meta
    res = {}
    for name, n in (('turn_sync_261', 261), ('part_counts_9', world + 1), ('block_sizes_4', 4)):
        t = torch.zeros(n, dtype=torch.int64)
        bufs = [torch.empty_like(t) for _ in range(world)]
        ts = []
        for i in range(rounds + 50):
            dist.barrier(group=meta)
            t0 = time.perf_counter()
            dist.all_gather(bufs, t, group=meta)
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts[50:]) * 1e6
        res[name] = {'median_us': round(float(np.median(ts)), 1), 'p90_us': round(float(np.percentile(ts, 90)), 1),
                     'mean_us': round(float(ts.mean()), 1)}
    # a back-to-back chain without barriers (the step's per-part gathers follow each other)
    t = torch.zeros(world + 1, dtype=torch.int64)
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.barrier(group=meta)
    t0 = time.perf_counter()
    for i in range(rounds):
        dist.all_gather(bufs, t, group=meta)
    res['part_counts_chain_us'] = round((time.perf_counter() - t0) / rounds * 1e6, 1)
    # the same gathers through shared memory (splendor_amd.dist.ShmMeta, the default when every rank is on one node)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'splendor-rl-gym_amd'))
    from splendor_amd.dist import ShmMeta
    shm = ShmMeta(rank, world, meta)
    for name, n in (('shm_turn_sync_261', 261), ('shm_part_counts_9', world + 1)):
        a = np.zeros(n, np.int64)
        ts = []
        for i in range(rounds + 50):
            dist.barrier(group=meta)
            t0 = time.perf_counter()
            shm.allgather(a)
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts[50:]) * 1e6
        res[name] = {'median_us': round(float(np.median(ts)), 1), 'p90_us': round(float(np.percentile(ts, 90)), 1),
                     'mean_us': round(float(ts.mean()), 1)}
    a = np.zeros(world + 1, np.int64)
    dist.barrier(group=meta)
    t0 = time.perf_counter()
    for i in range(rounds):
        shm.allgather(a)
    res['shm_part_counts_chain_us'] = round((time.perf_counter() - t0) / rounds * 1e6, 1)
    shm.close()
    all_res = [None] * world
    dist.all_gather_object(all_res, res)
    if rank == 0:
        with open(out, 'w') as f:
            json.dump(all_res, f)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=8)
    ap.add_argument('--rounds', type=int, default=400)
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, 'r.json')
        mp.spawn(worker, args=(a.world, _port(), a.rounds, f), nprocs=a.world, join=True)
        per = json.load(open(f))
    keys = [k for k in per[0] if isinstance(per[0][k], dict)]
    summary = {'world': a.world, 'rounds': a.rounds, 'host_cpus': os.cpu_count(),
               'all_gather': {k: {'median_us_max_rank': max(r[k]['median_us'] for r in per),
                                  'p90_us_max_rank': max(r[k]['p90_us'] for r in per)} for k in keys},
               'part_counts_chain_us_max_rank': max(r['part_counts_chain_us'] for r in per),
               'shm_part_counts_chain_us_max_rank': max(r['shm_part_counts_chain_us'] for r in per),
               'per_rank': per}
    print(json.dumps({k: v for k, v in summary.items() if k != 'per_rank'}, indent=1))
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(summary, f, indent=1)


if __name__ == '__main__':
    main()
