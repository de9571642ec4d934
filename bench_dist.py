"""bench.py --gpus N (N > 1): the sharded beam step, one process per GPU, RCCL over xGMI.

Launched by `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...` (bench.py starts
that launcher itself when run without one).  Weak scaling: every GPU holds --width states (global
beam_width = N x width; N=8 x 4M = 32M is config C5's width, heuristic `efficiency` by default).
As on one GPU, only the solve's saturated window is timed (queue full, no goal state: a probe solve
finds it, untimed), replayed on fresh seeded solves set up outside the timed region; each timed
segment is bracketed by barrier + device synchronize, the time is the max over ranks and
value = all parents expanded / that time.
"""
import json
import os
import random
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))


def keypass_pmc(kernel):
    """HBM bytes per step of the world > 1 key kernel (k_mkeys_a / k_keys_a) from the newest committed world-2
    serialised PMC summary (profiles/r*_w2_pmc.json, profiles/pmc_sharded.py), or None."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_w2_pmc.json')), reverse=True):
        try:
            v = json.load(open(f))['pmc'][kernel]
            return {'hbm_bytes_per_step': int(v['hbm_bytes_per_step']), 'device_ms_per_step': v['device_ms_per_step'],
                    'l2_hit_rate': v.get('tcc_hit_rate'),
                    'source': os.path.relpath(f, REPO) + ' (world 2 on one GPU, serialised ranks; rocprofv3 --pmc '
                              'FETCH_SIZE / WRITE_SIZE / TCC_HIT,MISS, separate passes; hbm = 2 FETCH + WRITE)'}
        except (KeyError, ValueError, OSError):
            continue
    return None


def carried_cpu_baseline():
    """The N=1 cpu_baseline measured by bench.py on a GPU box (profiles/r*_cpu_baseline_n1.json), carried on
    the N > 1 lines so every line has the CPU reference beside it (it is not re-timed there: the contract
    times it at N=1 only)."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_cpu_baseline_n1.json')), reverse=True):
        try:
            d = json.load(open(f))
            d['carried_from'] = os.path.relpath(f, REPO) + ' (measured at N=1 by bench.py on a GPU box host)'
            return d
        except (ValueError, OSError):
            continue
    return None


def sharded_pmc():
    """k_expand<true> (the sharded step's dominant kernel: own claims + records) from the newest committed
    sharded PMC summary (profiles/r*_profile_sharded_summary.json), or None."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_profile_sharded_summary.json')), reverse=True):
        try:
            d = json.load(open(f))
            v = d['pmc']['k_expand<true>']
            return {'kernel': 'k_expand<true>', 'hbm_bytes_per_launch': int(v['hbm_bytes_per_launch']),
                    'source': os.path.relpath(f, REPO) + ' (world 1, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)'}
        except (KeyError, ValueError, OSError):
            continue
    return None


def carried_n1(heuristic):
    """The N>1 lines' same-workload reference: `bench.py --gpus 1 --heuristic H` (the single-GPU engine at 4M per GPU)
    and the sharded protocol's world-1 run (SB_FORCE_DIST=1 SB_DIST_KP1=1: a rank's whole sharded device work on one
    GPU, nothing exchanged), both measured on a GPU box and committed under profiles/ (the newest round's)."""
    import glob
    out = {}
    for key, pat in (('single_gpu_engine', 'n1_{h}.json'), ('sharded_world1', 'n1_sharded_{h}.json')):
        fs = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'r*',
                                           pat.format(h=heuristic))))
        if not fs:
            continue
        try:
            d = json.load(open(fs[-1]))
        except (OSError, ValueError):
            continue
        out[key] = {'value': d['value'], 'ms_per_step': d['ms_per_step'], 'n_gpus': 1,
                    'source': os.path.relpath(fs[-1], os.path.dirname(os.path.abspath(__file__)))}
    if out:
        out['note'] = ('same workload (goal 15, -H ' + heuristic + ', 4M parents per GPU) on one MI355X, carried from the '
                       'committed run; scaling_efficiency = value / (n_gpus x the single-GPU engine\'s value)')
    return out or None


def main(args):
    # RCCL prints its version banner on stdout at init: keep stdout for the one JSON line
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    from bench import (GOAL, HBM_PEAK_GBS, METRIC, Window, cpu_baseline, expand_bytes, probe_window, step_bytes,
                       timed_steps, visited_summary)
    from splendor_amd.dist import Comm, DistSolve, HipBackend, SerializedBackend, TimedProxy
    from splendor_amd.engine import HEURISTIC_IDS
    if 'RANK' not in os.environ:   # SB_FORCE_DIST=1 without a launcher: a world of one
        os.environ.update(RANK='0', LOCAL_RANK='0', WORLD_SIZE='1', MASTER_ADDR='127.0.0.1',
                          MASTER_PORT=os.environ.get('MASTER_PORT', '29541'))
    backend = os.environ.get('SB_DIST_BACKEND', 'nccl')
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ndev = torch.cuda.device_count()
    # one GPU per rank; gloo (tests) or SB_DIST_SHARE_GPU=1 (probing RCCL on a one-GPU box) wrap ranks onto
    # the visible GPUs
    share = backend != 'nccl' or os.environ.get('SB_DIST_SHARE_GPU') == '1'
    dev = local % max(ndev, 1) if share else local
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, device_id=torch.device('cuda', dev) if backend == 'nccl' else None)
    rank, world = dist.get_rank(), dist.get_world_size()
    # distinct physical devices under this world: ranks share a GPU only when wrapped (gloo tests, share)
    n_phys = min(world, max(ndev, 1)) if share else world
    ranks_per_gpu = -(-world // n_phys)
    if world != args.gpus and not (args.gpus == 1 and os.environ.get('SB_FORCE_DIST') == '1'):
        raise RuntimeError(f'--gpus {args.gpus} but the launcher started a world of {world}')
    W = args.width * world
    serial = os.environ.get('SB_DIST_SERIALIZE') == '1' and world > 1
    hostprof = {} if os.environ.get('SB_DIST_HOSTPROF') == '1' else None

    bcs = []

    def make():
        random.seed(args.seed)
        b = HipBackend(rank=rank, world=world, device_index=dev, goal_pts=GOAL, use_heuristic=True,
                       heuristic=HEURISTIC_IDS[args.heuristic], beam_width=W, mt_state625=random.getstate()[1],
                       visited_log2=int(os.environ.get('SB_VISITED_LOG2', '0')),
                       extra_flags=int(os.environ.get('SB_DIST_FLAGS', '0')) | 1)   # 32: several ranks on one GPU;
        # 1: key-pass device time per step (the dominant world > 1 kernel's roofline); 256: card-set ownership
        comm = Comm(b.device)
        if serial:   # profiling several ranks on one GPU: each rank's device work alone (SerializedBackend),
            b = SerializedBackend(b)   # gloo's staging copies under the same lock
            comm.devlock = b.lock
        if hostprof is not None:   # host time inside each backend / collective call (SB_DIST_HOSTPROF=1)
            b, comm = TimedProxy(b, hostprof), TimedProxy(comm, hostprof)
        s = DistSolve(b, comm, goal_pts=GOAL, use_heuristic=True, beam_width=W)
        bcs.append(s.bc)
        return s

    vstats = []

    def close(s):
        vstats.append(s.b.visited_stats())   # this rank's owner shard: rebuilds short / skipped, peak load
        s.b.close()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()   # the exchange buffers of this solve go back to the device

    def sync_all(_s):
        torch.cuda.synchronize()
        dist.barrier()

    first, length, turns = probe_window(make, lambda s: s.step(), close, W)
    win = Window(make, lambda s: s.step(), lambda s: torch.cuda.synchronize(), close, first, length,
                 look=None if args.lookahead_edges else (lambda s, on: setattr(s, 'lookahead', on)))
    def sync_engine(_s):   # the timed turns' work (the engine runs on torch's stream); noise rounds ahead not waited for
        torch.cuda.current_stream().synchronize()

    per, el, el_eng, segs = timed_steps(win, args.steps, args.warmup, sync_all, sync_engine=sync_engine,
                                        engine_end=args.engine_stream_end,
                                        on_start=hostprof.clear if hostprof is not None else None)
    if hostprof is not None and rank == 0:   # the last timed segment's calls (cleared at each segment start)
        tot = sum(v[1] for v in hostprof.values())
        print(f'hostprof: last segment ({segs[-1]} steps; all segments {el * 1e3:.3f} ms wall over {len(per)} steps); '
              f'inside calls {tot * 1e3:.3f} ms', file=sys.stderr)
        for k, (c, t) in sorted(hostprof.items(), key=lambda kv: -kv[1][1]):
            print(f'hostprof {k:24s} calls {c:6d} ms {t * 1e3:9.3f}', file=sys.stderr)
    win.close()
    comm = Comm(torch.device('cuda', dev))
    el_max = float(comm.allreduce(np.array([int(el * 1e9)]), dist.ReduceOp.MAX)[0]) / 1e9
    el_eng_max = float(comm.allreduce(np.array([int(el_eng * 1e9)]), dist.ReduceOp.MAX)[0]) / 1e9
    parents = sum(p['n_parents'] for p in per)
    raw = sum(p['n_raw'] for p in per)
    uniq = sum(p['n_unique'] for p in per)
    kept = sum(p['n_kept'] for p in per)
    if rank == 0 and os.environ.get('SB_DIST_PHASES') == '1':
        for p in per:
            print('phases', p.get('phases'), file=sys.stderr, flush=True)
    if rank == 0:
        gbs = step_bytes(parents, raw, uniq, kept) / el_max / 1e9
        out = {
            'metric': METRIC, 'value': round(parents / el_max, 1), 'unit': 'states/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(el_max / args.steps * 1e3, 3),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u64+f64',
            'data': f'synthetic: seeded solve trajectory (random.seed({args.seed})); timed: the saturated turns '
                    f'{first}..{first + length - 1} of the {turns}-move goal-{GOAL} solve, replayed on '
                    f'{win.engines} seeded solves set up outside the timed region',
            'config': {'workload': f'speedrun goal_pts={GOAL} -u -H {args.heuristic} beam_width={W} '
                                   f'({args.width} per GPU; C5 at 8 GPUs x 4M)',
                       'beam_width': W, 'heuristic': args.heuristic, 'seed': args.seed,
                       'physical_gpus': n_phys, 'ranks_per_gpu': ranks_per_gpu, 'shared_gpu': ranks_per_gpu > 1,
                       'parallelism': (f'beam sharded over {world} ranks on {n_phys} GPU(s) ({backend}'
                                       + (f', {ranks_per_gpu} ranks per GPU: not a multi-GPU measurement' if ranks_per_gpu > 1
                                          else '') + '); trail owned by ')
                                      + ('card set (parents migrate to their owners; NOT bit-exact by construction: '
                                         'two card sets with an equal 64-bit key are both kept, DESIGN.md §6)'
                                         if world > 1 and (HipBackend.MIG or int(os.environ.get('SB_DIST_FLAGS', '0')) & 256)
                                         else 'key hash'),
                       'b_raw': round(raw / parents, 3), 'b_uniq': round(uniq / parents, 3),
                       'timed_turns': [first, first + length - 1], 'moves': turns,
                       'timed_expansions': ('engine lookahead at the window edges: the turn after each segment'
                                            if args.lookahead_edges else 'exactly the timed turns\' own'),
                       'segment_end': ('the engine stream (legacy: noise rounds for later turns not waited for)'
                                       if args.engine_stream_end else 'every stream + barrier'),
                       'segments': segs, 'warmup_engine': 'own (the timed steps start on fresh solves)',
                       'slices': ('block-cyclic: the next beam dealt in world x parts blocks, claims per part on arrival'
                                  if bcs and bcs[-1] else 'contiguous rank ranges'),
                       'visited_rank0': visited_summary(vstats[1:] or vstats)},
            'value_engine_stream_end': round(parents / el_eng_max, 1),
            # bytes rank 0 sent to other ranks per timed step, by exchange (Comm.acct; RCCL's own traffic)
            'exchange_MB_per_step_rank0': {k: round(sum(p.get('xbytes', {}).get(k, 0) for p in per) / len(per) / 1e6, 2)
                                           for k in sorted({k for p in per for k in p.get('xbytes', {})})},
            # collectives rank 0 issued per timed step: device-group rounds (RCCL's latency terms) and host metadata
            # all_gathers (shared memory on one node) — counted by Comm, not assumed
            'collectives_per_step_rank0': {
                'device': round(sum(p.get('collectives', (0, 0))[0] for p in per) / len(per), 2),
                'host': round(sum(p.get('collectives', (0, 0))[1] for p in per) / len(per), 2)},
            'roofline': {'bound': 'hbm', 'kernel': 'whole step (per GPU, SURVEY §8d byte model)',
                         'achieved': round(gbs / world, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(gbs / world / HBM_PEAK_GBS, 5), 'traffic': None},
            'cpu_baseline': None,
        }
        kp = [p['keypass_ms'] for p in per if p.get('keypass_ms')]
        if world > 1 and kp:
            # the dominant world > 1 kernel: the key pass (k_mkeys_a with card-set ownership, else k_keys_a), its
            # device time per step from HIP events around its launches on this rank (rank 0), its algorithmic
            # bytes per rank: 16 B parent + 24 B masks + 21 B per raw child + 16 B per new key (bench.py's
            # expand_bytes, the single GPU's k_expand model), at the all-rank mean share (raw / world ...)
            mig_on = HipBackend.MIG or bool(int(os.environ.get('SB_DIST_FLAGS', '0')) & 256)
            kname = 'k_mkeys_a' if mig_on else 'k_keys_a'
            kms = sum(kp) / len(kp)
            abytes = expand_bytes(parents / len(per) / world, raw / len(per) / world, uniq / len(per) / world)
            ach = abytes / (kms * 1e-3) / 1e9
            out['roofline'] = {'bound': 'hbm', 'kernel': kname, 'achieved': round(ach, 2), 'peak': HBM_PEAK_GBS,
                               'unit': 'GB/s', 'frac': round(ach / HBM_PEAK_GBS, 5), 'traffic': None,
                               'launch_ms': round(kms, 4), 'launches_per_step': int(os.environ.get('SB_DIST_PARTS', '4')),
                               'algorithmic_bytes_per_step': int(abytes),
                               'whole_step': {'model': 'SURVEY §8d per GPU', 'achieved': round(gbs / world, 2),
                                              'frac': round(gbs / world / HBM_PEAK_GBS, 5)}}
            if ranks_per_gpu > 1:   # the launch time includes the other ranks' work on the same device
                out['roofline']['per_gpu_valid'] = False
                out['roofline']['note'] = (f'{ranks_per_gpu} ranks share each GPU: the key kernel\'s event time '
                                           'includes contention from the other ranks, so this is not a per-GPU roofline')
            pm = keypass_pmc(kname)
            if pm:
                out['roofline']['traffic'] = pm['hbm_bytes_per_step']
                out['roofline']['traffic_device_ms'] = round(pm['device_ms_per_step'], 4)
                out['roofline']['l2_hit_rate'] = pm['l2_hit_rate']
                out['roofline']['traffic_source'] = pm['source']
        else:
            sh = sharded_pmc()
            if sh:   # the dominant kernel's HBM bytes per launch, profiled on the sharded path at world 1
                out['roofline']['traffic'] = sh['hbm_bytes_per_launch']
                out['roofline']['traffic_kernel'] = sh['kernel']
                out['roofline']['traffic_source'] = sh['source']
        if world > 1:   # the same workload on one GPU, measured on a GPU box and carried
            n1 = carried_n1(args.heuristic)
            if n1:
                out['n1_same_workload'] = n1
                if n1.get('single_gpu_engine'):
                    out['scaling_efficiency'] = round(out['value'] / (world * n1['single_gpu_engine']['value']), 4)
        if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only, after the timed region
            out['cpu_baseline'] = cpu_baseline(args.width, args.heuristic, args.seed, first)
        elif world > 1:
            out['cpu_baseline'] = carried_cpu_baseline()
        sys.stdout.flush()
        os.dup2(json_fd, 1)
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
