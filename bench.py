#!/usr/bin/env python3
"""Benchmark: states expanded/sec per beam step (BASELINE.json metric) on MI355X.

Workload (N=1): config C3 of BASELINE.json — speedrun goal 15, -u -H balanced, beam_width 4,000,000,
random.seed(0) (the largest single-GPU config; C2 at W=300k is a parity case, not a bench line).
The engine runs the seeded solve from the root; the steps until the beam first fills (turns 0..8)
are setup, then `--warmup` untimed steps, then exactly `--steps` timed steps.  A step is one full
sb_step: goal check, expansion + hash + visited claim, survivor check, next_queue scan, state/score
emission with MT19937 noise, stable top-k, beam write.  The goal is raised to 255 for the timing run
so that more than the 6 saturated turns of the goal-15 trajectory can be timed; up to turn 15 the
trajectory is identical to the goal-15 solve (the goal is first reached at turn 15).

Output: one JSON line (rank 0) with `roofline` for the dominant kernel (device events on the engine's
stream) and `cpu_baseline` (the C oracle, single thread, same config and seed, bounded sample).
"""
import argparse
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'splendor-rl-gym_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))

METRIC = 'states expanded/sec per beam step, goal=15 beam_width=4M, 1/2/4/8 MI355X'
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
RANDOM_LOAD_PEAK_G = 48.0   # random 16-B loads / s over a 32 GiB table, measured (profiles/micro/r1_randaccess.txt)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--width', type=int, default=4_000_000)
    ap.add_argument('--heuristic', default='balanced')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-budget-s', type=float, default=30.0)
    ap.add_argument('--realistic', action='store_true',
                    help='config C4 instead: realistic 2-player goal 15 --shuffle, W=1M (a separate line, not the '
                         'headline metric)')
    return ap.parse_args()


# algorithmic bytes of k_expand per parent: parent 16 B read; per raw child a 16 B
# visited-entry read, a 4 B slot + 1 B desc write; per candidate child an 8 B claim (atomicMin)
# and, for new keys, an 8 B key CAS; per parent the 24 B candidate mask.
def expand_bytes(n_parents, n_raw, n_cand_new):
    return 16 * n_parents + 21 * n_raw + 16 * n_cand_new + 24 * n_parents


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary (profiles/)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_profile_summary.json')))
    for f in reversed(files):
        try:
            d = json.load(open(f))
            v = d['pmc'][kernel]['hbm_bytes_per_launch']
            t = d['timed'][kernel]['avg_ns']
            return v, t, os.path.relpath(f, REPO)
        except (KeyError, ValueError, OSError):
            continue
    return None, None, None


def step_bytes(n_parents, n_raw, n_unique, n_kept):
    """SURVEY.md §8(d) whole-step model: 28 + 20 b_raw + 37 b_uniq + 33 per parent (with our 16 B state)."""
    return 28 * n_parents + 20 * n_raw + 37 * n_unique + 33 * n_kept


def cpu_baseline(width, heuristic, seed, budget_s):
    """C oracle (single thread) on the same seeded trajectory, bounded: turns run until the budget."""
    import oracle_c
    random.seed(seed)
    st = random.getstate()[1]
    o = oracle_c.OracleSolve(255, use_heuristic=True, heuristic_name=heuristic, beam_width=width, mt_state625=st)
    t_start = time.perf_counter()
    best = None
    turn = 0
    while True:
        t0 = time.perf_counter()
        r = o.step()
        dt = time.perf_counter() - t0
        if r['n_parents'] >= 100_000:
            best = (turn, r['n_parents'], dt)
        turn += 1
        if r['done'] or r['n_parents'] >= width:
            break
        # next step's cost ~ dt * growth of the queue; stop before it would overrun the budget
        growth = r['n_kept'] / max(r['n_parents'], 1)
        if (time.perf_counter() - t_start) + dt * growth > budget_s:
            break
    o.close()
    if best is None:
        return None
    t, n, dt = best
    return {'value': round(n / dt, 1), 'unit': 'states/s', 'cores': 1, 'kind': 'port',
            'sample': f'C oracle (oracle/csrc/oracle.c), 1 thread, same config and seed; turn {t} '
                      f'({n} parents) of the W={width} trajectory, {dt:.2f} s; host cores '
                      f'available {len(os.sched_getaffinity(0))}'}


def run_single(args):
    from splendor_amd.engine import HEURISTIC_IDS, BeamEngine
    random.seed(args.seed)
    st = random.getstate()[1]
    eng = BeamEngine(goal_pts=255, use_heuristic=True, heuristic=HEURISTIC_IDS[args.heuristic],
                     beam_width=args.width, mt_state625=st, device=0, timing=True)
    setup_turns = 0
    while True:   # setup: until the beam is full
        r = eng.step()
        setup_turns += 1
        if r['n_kept'] >= args.width or r['done']:
            break
    for _ in range(args.warmup):
        eng.step()
    eng.sync()
    per = []
    turn0 = eng.turn
    t0 = time.perf_counter()
    for _ in range(args.steps):
        per.append(eng.step())
    eng.sync()
    elapsed = time.perf_counter() - t0
    # device phase times of the timed turns (HIP events recorded on the engine's stream)
    for i, p in enumerate(per):
        p.update(eng.turn_times(turn0 + i))
    eng.close()
    return per, elapsed, setup_turns


def run_realistic(args):
    """Config C4: MultiPlayerState beam search, 2 players, goal 15, shuffled market (seed 0), W=1M."""
    from splendor_amd.engine_rt import RealisticEngine
    from splendor_amd.realistic import GameConfig, MultiPlayerState
    width = args.width if args.width != 4_000_000 else 1_000_000
    cfg = GameConfig(num_players=2, target_points=15, gems_per_color=4, infinite_resources=False)
    root = MultiPlayerState.newgame(config=cfg, shuffle_market=True, seed=args.seed)
    random.seed(args.seed)
    eng = RealisticEngine(root, beam_width=width, mt_state625=random.getstate()[1], device=0)
    setup = 0
    while True:
        r = eng.step()
        setup += 1
        if r['n_kept'] >= width or r['done']:
            break
    for _ in range(args.warmup):
        eng.step()
    import ctypes
    from splendor_amd import _lib
    _lib.lib().sb_sync(eng._h)
    per = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        per.append(eng.step())
        if per[-1]['done']:
            break
    _lib.lib().sb_sync(eng._h)
    elapsed = time.perf_counter() - t0
    eng.close()
    parents = sum(p['n_parents'] for p in per)
    out = {'metric': 'states expanded/sec per beam step, realistic 2-player goal 15 --shuffle, beam_width=1M',
           'value': round(parents / elapsed, 1), 'unit': 'states/s', 'n_gpus': 1, 'steps': len(per),
           'warmup': args.warmup, 'ms_per_step': round(elapsed / len(per) * 1e3, 3), 'higher_is_better': True,
           'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u64+f64',
           'data': f'synthetic: seeded realistic solve trajectory (market shuffle seed {args.seed}, random.seed('
                   f'{args.seed})), saturated turns {setup + args.warmup}..{setup + args.warmup + len(per) - 1}',
           'config': {'workload': f'realistic 2p goal_pts=15 --shuffle beam_width={width} (C4)', 'beam_width': width,
                      'b_raw': round(sum(p['n_raw'] for p in per) / parents, 3),
                      'b_uniq': round(sum(p['n_unique'] for p in per) / parents, 3)}}
    print(json.dumps(out))


def main():
    args = parse()
    if args.realistic:
        return run_realistic(args)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world > 1 or args.gpus > 1 or os.environ.get('SB_FORCE_DIST') == '1':   # (diagnostic: sharded path at N=1)
        import bench_dist
        return bench_dist.main(args)
    per, elapsed, setup_turns = run_single(args)
    parents = sum(p['n_parents'] for p in per)
    raw = sum(p['n_raw'] for p in per)
    uniq = sum(p['n_unique'] for p in per)
    kept = sum(p['n_kept'] for p in per)
    phases = {k: round(sum(p[k] for p in per) / len(per), 3) for k in
              ('ms_expand', 'ms_survive', 'ms_mt', 'ms_emit', 'ms_select', 'ms_gather', 'ms_total')}
    dom = max(('ms_expand', 'ms_survive', 'ms_emit', 'ms_select', 'ms_gather'), key=lambda k: phases[k])
    # roofline of the dominant phase (k_expand in practice): algorithmic bytes / its device time
    ms_dom = phases[dom]
    n_par = parents / len(per)
    if dom == 'ms_expand':
        byt = expand_bytes(n_par, raw / len(per), uniq / len(per))
    else:
        byt = step_bytes(n_par, raw / len(per), uniq / len(per), kept / len(per)) * 0.25
    achieved = byt / (ms_dom * 1e-3) / 1e9 if ms_dom > 0 else 0.0
    out = {
        'metric': METRIC,
        'value': round(parents / elapsed, 1),
        'unit': 'states/s',
        'n_gpus': 1,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'u64+f64',
        'data': f'synthetic: seeded solve trajectory (random.seed({args.seed})), saturated turns '
                f'{setup_turns + args.warmup}..{setup_turns + args.warmup + args.steps - 1}',
        'config': {'workload': f'speedrun goal_pts=15 -u -H {args.heuristic} beam_width={args.width} (C3)',
                   'beam_width': args.width, 'heuristic': args.heuristic, 'seed': args.seed,
                   'parallelism': 'single GPU', 'b_raw': round(raw / parents, 3), 'b_uniq': round(uniq / parents, 3)},
        'phases_ms': phases,
        'roofline': {'bound': 'hbm', 'kernel': dom.replace('ms_', 'k_'), 'achieved': round(achieved, 2),
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 5),
                     'algorithmic_bytes_per_launch': int(byt), 'launch_ms': ms_dom, 'traffic': None},
        'step_model_GBps': round(step_bytes(parents, raw, uniq, kept) / elapsed / 1e9, 2),
        'cpu_baseline': None,
    }
    if dom == 'ms_expand':
        # the bound that actually binds k_expand: random 128-B line requests — one probe
        # load per raw child and one tag CAS per new key (= per survivor; its key store follows on the
        # same line), lost marks not counted (a lower bound) — against the measured random 16-B load
        # rate over a 32 GiB table
        touches = (raw + uniq) / len(per)
        out['roofline']['random_access'] = {
            'touches_per_launch': int(touches), 'achieved_G_per_s': round(touches / (ms_dom * 1e-3) / 1e9, 2),
            'peak_G_per_s': RANDOM_LOAD_PEAK_G, 'frac': round(touches / (ms_dom * 1e-3) / 1e9 / RANDOM_LOAD_PEAK_G, 3),
            'peak_source': 'profiles/micro/r1_randaccess.txt (load16, 32 GiB table)'}
    tr, tns, src = pmc_traffic(dom.replace('ms_', 'k_'))
    if tr is not None:
        out['roofline']['traffic'] = int(tr)
        out['roofline']['traffic_GBps'] = round(tr / (tns * 1e-9) / 1e9, 1)
        out['roofline']['traffic_source'] = f'{src} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; ' \
                                            f'hbm = (2*FETCH + WRITE) KiB, gfx950 correction)'
    if not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(args.width, args.heuristic, args.seed, args.cpu_budget_s)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
