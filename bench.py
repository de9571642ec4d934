#!/usr/bin/env python3
"""Benchmark: states expanded/sec per beam step (BASELINE.json metric) on MI355X.

Workload (N=1): config C3 of BASELINE.json — speedrun goal 15, -u -H balanced, beam_width 4,000,000,
random.seed(0) (the largest single-GPU config; C2 at W=300k is a parity case, not a bench line).

Only C3's own saturated steps are timed.  A probe solve (untimed, also the warmup) finds the window:
the steps whose queue is full (n_parents == W) and holds no goal state, i.e. turns 9..14 of the seeded
goal-15 trajectory (the goal check of turn 15 ends the solve, src/solver.py:438-445).  `--steps K`
beyond one window replays it: a fresh engine with the same seed is set up outside the timed region
(turns 0..8) and its window is timed again.  Every timed segment is bracketed by a device sync (and a
barrier with N > 1); `ms_per_step` = the summed segment time / K.  A step is one full sb_step: goal
check, expansion + hash + visited claim, survivor count, next_queue scan, state/score emission with
MT19937 noise, stable top-k, beam write (the expansion of the next queue is pipelined behind the gather,
so a timed window of turns t..u covers the expansions of queues t+1..u+1).

--gpus N > 1: one process per GPU over RCCL (bench_dist.py, the sharded step).  Without a launcher
environment the script starts `torch.distributed.run` itself (before any GPU call) and exits with its
return code.

Output: one JSON line (rank 0) with `roofline` for the dominant kernel (device events on the engine's
stream) and `cpu_baseline` (the C oracle, single thread, same config and seed, bounded sample).
"""
import argparse
import json
import os
import random
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'splendor-rl-gym_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))

METRIC = 'states expanded/sec per beam step, goal=15 beam_width=4M, 1/2/4/8 MI355X'
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
RANDOM_LOAD_PEAK_G = 48.0   # random 16-B loads / s over a 32 GiB table, measured (profiles/micro/r1_randaccess.txt)
RANDOM_PROBE_G = 45.46    # random 16-B loads over a 32 GiB table (profiles/micro/fetchcal.hip, round 4)
RANDOM_INSERT_G = 19.07   # probe + tag CAS + key store on one random line (same micro)
GOAL = 15                   # C3 / C5 goal_pts
# the reference's own CPU path on C3's heuristic, measured in the build container (BASELINE.md §2 / SURVEY §6):
# pure Python, 1 core; it cannot run on the GPU box (the reference does not travel), so it is quoted, not timed
PY_REFERENCE = {'balanced': (11421, 'goal 15 -u -H balanced W=1M, saturated step 87.6 s'),
                'efficiency': (8323, 'goal 15 -u -H efficiency W=300k, saturated step 36.0 s (3 runs sharing 8 cores)'),
                'simple': (13093, 'goal 15 -u -H simple W=300k, saturated step 22.9 s')}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=12)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--width', type=int, default=4_000_000, help='beam width per GPU')
    ap.add_argument('--heuristic', default=None,
                    help='default: balanced (C3) on one GPU, efficiency (C5) on the sharded path')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--dry-run', action='store_true',
                    help='launcher plumbing only (CPU, gloo): every rank joins the group, rank 0 prints the world; '
                         'no GPU call (tests/test_bench_launch.py)')
    ap.add_argument('--lookahead-edges', action='store_true',
                    help='time the window with the engine lookahead at its edges too (the first timed turn\'s '
                         'expansion runs before the clock starts, the turn after the window\'s inside it)')
    ap.add_argument('--engine-stream-end', action='store_true',
                    help='legacy accounting: end each timed segment when the engine stream is idle, not waiting '
                         'for the noise generation that runs ahead for later turns on its own stream')
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
    """(HBM bytes per launch, trace average ns, L2 hit rate, source) of `kernel` (or its template instance
    used by this path, e.g. k_expand<false>) from the newest committed rocprofv3 PMC summary (profiles/)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_profile_summary.json')))
    for f in reversed(files):
        try:
            d = json.load(open(f))
            name = next(k for k in d['pmc'] if k == kernel or k == kernel + '<false>')
            v = d['pmc'][name]['hbm_bytes_per_launch']
            t = d['timed'][name]['avg_ns']
            return v, t, d['pmc'][name].get('tcc_hit_rate'), os.path.relpath(f, REPO)
        except (KeyError, ValueError, OSError, StopIteration):
            continue
    return None, None, None, None


def step_bytes(n_parents, n_raw, n_unique, n_kept):
    """SURVEY.md §8(d) whole-step model: 28 + 20 b_raw + 37 b_uniq + 33 per parent (with our 16 B state)."""
    return 28 * n_parents + 20 * n_raw + 37 * n_unique + 33 * n_kept


def cpu_baseline(width, heuristic, seed, first_turn, py_sample=100_000):
    """The CPU path on this box's host cores, single thread, same config and seed (VERDICT r2 missing 2,
    r4 weak 8): the C oracle brings the bench config's own solve (W = width) to the GPU's first timed turn,
    untimed; `value` = the pure-Python restatement of the reference's step (oracle/pyref.py: CPython objects,
    tuple hash, set trail, random.randint, stable sorted — the reference's own CPU path, which cannot travel
    here) timed on a bounded sample of that turn (its first py_sample parents); `c_oracle` = the C port
    (oracle/csrc/oracle.c) timed on the whole turn."""
    import oracle_c
    import pyref
    out = {}
    random.seed(seed)
    o = oracle_c.OracleSolve(255, use_heuristic=True, heuristic_name=heuristic, beam_width=width,
                             mt_state625=random.getstate()[1])
    t0 = time.perf_counter()
    for _ in range(first_turn):
        o.step()
    setup = time.perf_counter() - t0
    turn = o.nturns() - 1
    # pure Python: a bounded sample of the first timed turn (its first py_sample parents)
    ps = pyref.from_oracle(o, 255, heuristic, width, sample=py_sample)
    t0 = time.perf_counter()
    r = ps.step()
    dt = time.perf_counter() - t0
    del ps
    out.update(value=round(r['n_parents'] / dt, 1), unit='states/s', cores=1, kind='port',
               label='pure-Python port of the reference step on a sample of the GPU\'s first timed turn '
                     '(python_reference_quoted below is the reference itself, on a W=1M saturated step)',
               sample=f'pure-Python restatement of the reference step (oracle/pyref.py, CPython '
                      f'{sys.version.split()[0]}, 1 thread) on the GPU\'s first timed turn of this config '
                      f'(-H {heuristic}, W={width}, seed {seed}: the beam after turn {turn}), its first '
                      f'{r["n_parents"]} parents ({r["n_raw"]} children, {r["n_unique"]} new against a trail of '
                      f'that beam\'s keys), {dt:.2f} s; host cores available {len(os.sched_getaffinity(0))}')
    # C port on the whole first timed turn
    t0 = time.perf_counter()
    r = o.step()
    dt = time.perf_counter() - t0
    o.close()
    out['c_oracle'] = {'value': round(r['n_parents'] / dt, 1), 'unit': 'states/s', 'cores': 1, 'kind': 'port',
                       'sample': f'C oracle (oracle/csrc/oracle.c), 1 thread: turn {first_turn} of the W={width} '
                                 f'trajectory (the first timed turn, {r["n_parents"]} parents), {dt:.2f} s '
                                 f'(setup turns {setup:.1f} s, untimed)'}
    if heuristic in PY_REFERENCE:
        v, what = PY_REFERENCE[heuristic]
        out['python_reference_quoted'] = {
            'value': v, 'unit': 'states/s', 'cores': 1,
            'source': f'the reference itself (src/solver.py, CPython 3.10) on {what}, measured in the build '
                      'container (BASELINE.md §2): the reference cannot travel to the GPU box'}
    return out


class Window:
    """Feeds the timed loop with C3-window steps: each engine is set up (untimed) from the root with the
    same seed up to the first saturated turn; `left` steps of its window remain.  `make()` builds a
    seeded engine; `step(e)` / `sync(e)` / `close(e)` drive it."""

    def __init__(self, make, step, sync, close, first, length, look=None):
        self.make, self._step, self._sync, self._close = make, step, sync, close
        self.look = look   # look(e, on): sb_set_lookahead (None: the engine always launches ahead)
        self.first, self.length = first, length   # window turns first .. first+length-1
        self.eng, self.left, self.engines = None, 0, 0

    def ensure(self):
        if self.left > 0:
            return
        if self.eng is not None:
            self._close(self.eng)
            self.eng = None
        self.eng = self.make()
        self.engines += 1
        for t in range(self.first):   # setup: turns 0 .. first-1
            if self.look and t == self.first - 1:   # the first window turn's expansion is timed with it
                self.look(self.eng, False)
            t0 = time.perf_counter()
            r = self._step(self.eng)
            _progress(f'setup turn {t}', t0)
            assert not r['done'], 'setup reached the goal'
        if self.look:
            self.look(self.eng, True)
        self.left = self.length
        self._sync(self.eng)

    def step(self):
        self.left -= 1
        r = self._step(self.eng)
        assert not r['done'], 'stepped past the window'
        return r

    def close(self):
        if self.eng is not None:
            self._close(self.eng)
            self.eng = None


PROGRESS = os.environ.get('SB_BENCH_PROGRESS') == '1'   # a line per step on stderr (long profiled runs)


def _progress(what, t0):
    if PROGRESS:
        print(f'[bench] {what} {time.perf_counter() - t0:.3f} s', file=sys.stderr, flush=True)


def probe_window(make, step, close, width):
    """Run one seeded solve to its goal: (first saturated turn, window length, turns, moves).  The window
    is the steps whose queue is full and has no goal state (every later step of the solve ends it)."""
    eng = make()
    turn, first, last = 0, None, None
    while True:
        t0 = time.perf_counter()
        r = step(eng)
        _progress(f'probe turn {turn}', t0)
        if r['done']:
            break
        if r['n_parents'] >= width and first is None:
            first = turn
        if first is not None:
            last = turn
        turn += 1
    close(eng)
    if first is None:
        raise RuntimeError('the beam never saturates before the goal: nothing to time')
    return first, last - first + 1, turn


def timed_steps(win, steps, warmup, sync_all, on_segment=None, sync_engine=None, engine_end=False, on_start=None):
    """Warmup on an engine of its own, then exactly `steps` timed window steps on fresh engines, segment by
    segment (a segment ends where an engine's window ends).  Each segment starts with every stream idle
    and ends with every stream synced (the noise generated inside it for later turns is charged to it);
    `sync_engine`, when given, also notes when the engine stream alone finished.  `engine_end` (legacy
    accounting) stops the clock there instead.  Returns (per-step stats, seconds, engine-stream seconds,
    segment lengths)."""
    for _ in range(warmup):
        win.ensure()
        win.step()
    win.left = 0   # the timed steps start on a fresh engine
    per, total, total_eng, segs = [], 0.0, 0.0, []
    while len(per) < steps:
        win.ensure()
        n = min(steps - len(per), win.left)
        turn0 = win.first + win.length - win.left
        sync_all(win.eng)
        if on_start:
            on_start()
        t0 = time.perf_counter()
        seg = []
        for i in range(n):
            if win.look and i == n - 1:   # the segment's last step does not start the next turn's expansion
                win.look(win.eng, False)
            seg.append(win.step())
        if sync_engine:
            sync_engine(win.eng)
        t_eng = time.perf_counter() - t0
        if not engine_end:
            sync_all(win.eng)
        dt = time.perf_counter() - t0
        total += dt
        total_eng += t_eng
        segs.append(n)
        if win.look:
            win.look(win.eng, True)
        if on_segment:
            on_segment(win.eng, turn0, seg)
        _progress(f'timed segment of {n} steps', t0)
        if os.environ.get('SB_BENCH_SEGDBG'):
            ev = sum(p.get('ms_total', 0.0) for p in seg)
            print(f'segment turns {turn0}..{turn0 + n - 1}: wall {dt * 1e3:.3f} ms (engine stream {t_eng * 1e3:.3f}), '
                  f'device events {ev:.3f} ms', file=sys.stderr, flush=True)
        per += seg
    return per, total, total_eng, segs


def run_single(args):
    from splendor_amd.engine import HEURISTIC_IDS, BeamEngine
    heur = args.heuristic

    def make():
        random.seed(args.seed)
        return BeamEngine(goal_pts=GOAL, use_heuristic=True, heuristic=HEURISTIC_IDS[heur],
                          beam_width=args.width, mt_state625=random.getstate()[1], device=0, timing=True)

    first, length, turns = probe_window(make, lambda e: e.step(), lambda e: e.close(), args.width)
    win = Window(make, lambda e: e.step(), lambda e: e.sync(), lambda e: e.close(), first, length,
                 look=None if args.lookahead_edges else (lambda e, on: e.set_lookahead(on)))

    vstats = []

    def phases(eng, turn0, seg):   # device phase times (HIP events recorded on the engine's stream)
        for i, p in enumerate(seg):
            p.update(eng.turn_times(turn0 + i))
        vstats.append(eng.visited_stats())   # the visited set's growth record (shortened / skipped rebuilds)

    # the clock stops when every stream is idle: the MT producers' chunk that the segment's last step
    # launched for later turns is charged to the segment (--engine-stream-end: legacy accounting that
    # stops at the engine stream; its figure is reported beside `value` either way)
    per, elapsed, el_eng, segs = timed_steps(win, args.steps, args.warmup, lambda e: e.sync(), phases,
                                             sync_engine=lambda e: e.sync_engine(), engine_end=args.engine_stream_end)
    win.close()
    return per, elapsed, el_eng, segs, (first, length, turns, win.engines), visited_summary(vstats)


def visited_summary(vstats):
    """The timed engines' visited sets: slots at the end, rebuilds, rebuilds short of the worst case or skipped (free
    HBM ran short: a higher load and longer probe chains, never a different result), the peak load after a turn."""
    if not vstats:
        return None
    return {'slots': max(v['slots'] for v in vstats), 'rebuilds': max(v['rebuilds'] for v in vstats),
            'rebuilds_short': sum(v['rebuilds_short'] for v in vstats),
            'rebuilds_skipped': sum(v['rebuilds_skipped'] for v in vstats),
            'peak_load': max(v['peak_load'] for v in vstats)}


def rexpand_bytes(n_parents, n_raw, n_unique):
    """Algorithmic bytes of k_rexpand2 per launch: the parent's 12-word state (96 B) and its
    24 B of candidate / lost masks; per raw child a 16 B visited-entry probe; per new key an 8 B tag CAS
    and an 8 B key store."""
    return 120 * n_parents + 16 * n_raw + 16 * n_unique


def cpu_baseline_realistic(width, seed, first_turn):
    """The realistic C oracle (oracle/csrc/oracle.c, ort_*), 1 thread, on the first timed turn of the same
    seeded C4 trajectory (setup turns untimed)."""
    import numpy as np
    import oracle_c
    from splendor_amd.engine_rt import device_tiers
    from splendor_amd.realistic import GameConfig, MultiPlayerState, game_params, pack_state
    cfg = GameConfig(num_players=2, target_points=15, gems_per_color=4, infinite_resources=False)
    root = MultiPlayerState.newgame(config=cfg, shuffle_market=True, seed=seed)
    tiers0 = device_tiers(root)
    params, tiers = game_params(cfg, tiers0)
    random.seed(seed)
    o = oracle_c.OracleRealistic(params, tiers, beam_width=width, mt_state625=random.getstate()[1],
                                 root_w=np.asarray(pack_state(root, tiers0)))
    for _ in range(first_turn):
        o.step()
    t0 = time.perf_counter()
    r = o.step()
    dt = time.perf_counter() - t0
    o.close()
    return {'value': round(r['n_parents'] / dt, 1), 'unit': 'states/s', 'cores': 1, 'kind': 'port',
            'sample': f'realistic C oracle (oracle/csrc/oracle.c ort_step), 1 thread: turn {first_turn} of the C4 '
                      f'trajectory ({r["n_parents"]} parents), {dt:.2f} s; host cores available '
                      f'{len(os.sched_getaffinity(0))}',
            'python_reference_quoted': {'value': 3600, 'unit': 'states/s', 'cores': 1,
                                        'source': 'the reference itself (MultiPlayerState.solve), SURVEY.md §8(a) '
                                                  'a12, measured in the build container'}}


def run_realistic(args):
    """Config C4: MultiPlayerState beam search, 2 players, goal 15, shuffled market (seed 0), W=1M."""
    from splendor_amd.engine_rt import RealisticEngine
    from splendor_amd.realistic import GameConfig, MultiPlayerState
    width = args.width if args.width != 4_000_000 else 1_000_000
    cfg = GameConfig(num_players=2, target_points=15, gems_per_color=4, infinite_resources=False)

    def make():
        root = MultiPlayerState.newgame(config=cfg, shuffle_market=True, seed=args.seed)
        random.seed(args.seed)
        return RealisticEngine(root, beam_width=width, mt_state625=random.getstate()[1], device=0, timing=True)

    from splendor_amd import _lib
    sync = lambda e: _lib.lib().sb_sync(e._h)
    first, length, turns = probe_window(make, lambda e: e.step(), lambda e: e.close(), width)
    win = Window(make, lambda e: e.step(), sync, lambda e: e.close(), first, length)

    vstats = []

    def phases(eng, turn0, seg):
        for i, p in enumerate(seg):
            p.update(eng.turn_times(turn0 + i))
        vstats.append(eng.visited_stats())

    per, elapsed, _, segs = timed_steps(win, args.steps, args.warmup, sync, phases)
    win.close()
    parents = sum(p['n_parents'] for p in per)
    raw = sum(p['n_raw'] for p in per)
    uniq = sum(p['n_unique'] for p in per)
    K = len(per)
    ph = {k: round(sum(p[k] for p in per) / K, 3) for k in
          ('ms_expand', 'ms_survive', 'ms_mt', 'ms_emit', 'ms_select', 'ms_gather', 'ms_total')}
    byt = rexpand_bytes(parents / K, raw / K, uniq / K)
    achieved = byt / (ph['ms_expand'] * 1e-3) / 1e9 if ph['ms_expand'] > 0 else 0.0
    out = {'metric': 'states expanded/sec per beam step, realistic 2-player goal 15 --shuffle, beam_width=1M',
           'value': round(parents / elapsed, 1), 'unit': 'states/s', 'n_gpus': 1, 'steps': K,
           'warmup': args.warmup, 'ms_per_step': round(elapsed / K * 1e3, 3), 'higher_is_better': True,
           'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u64+f64',
           'data': f'synthetic: seeded realistic solve trajectory (market shuffle seed {args.seed}, random.seed('
                   f'{args.seed})); timed: saturated turns {first}..{first + length - 1} of the {turns}-move game, '
                   f'replayed on {win.engines} seeded engines',
           'config': {'workload': f'realistic 2p goal_pts=15 --shuffle beam_width={width} (C4)', 'beam_width': width,
                      'b_raw': round(raw / parents, 3), 'b_uniq': round(uniq / parents, 3),
                      'segment_end': 'every stream', 'segments': segs,
                      'warmup_engine': 'own (the timed steps start on fresh engines)',
                      'visited': visited_summary(vstats)},
           'phases_ms': ph,
           'roofline': {'bound': 'hbm', 'kernel': 'k_rexpand2', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS,
                        'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 5),
                        'algorithmic_bytes_per_launch': int(byt), 'launch_ms': ph['ms_expand'], 'traffic': None},
           'cpu_baseline': None}
    tr, tns, hit, src = pmc_traffic('k_rexpand2<1>')
    if tr is not None:
        out['roofline']['traffic'] = int(tr)
        out['roofline']['traffic_GBps'] = round(tr / (tns * 1e-9) / 1e9, 1)
        if hit is not None:
            out['roofline']['l2_hit_rate'] = round(hit, 4)
        out['roofline']['traffic_source'] = f'{src} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; ' \
                                            f'hbm = (2*FETCH + WRITE) KiB, gfx950 correction)'
    if not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline_realistic(width, args.seed, first)
    print(json.dumps(out))


def self_launch(args):
    """--gpus N > 1 without a launcher: one process per GPU via torch.distributed.run (child process; the
    parent has not touched the GPU), exit with its code."""
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr=127.0.0.1', f'--master-port={port}', os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, SB_BENCH_LAUNCHED='1')
    return subprocess.call(cmd, env=env)


def dry_run(args):
    import torch.distributed as dist
    if 'RANK' not in os.environ:
        os.environ.update(RANK='0', LOCAL_RANK='0', WORLD_SIZE='1', MASTER_ADDR='127.0.0.1', MASTER_PORT='29542')
    dist.init_process_group('gloo')
    world = dist.get_world_size()
    if world != args.gpus:
        raise RuntimeError(f'--gpus {args.gpus} but the launcher started a world of {world}')
    dist.barrier()
    if dist.get_rank() == 0:
        print(json.dumps({'metric': METRIC, 'n_gpus': world, 'dry_run': True,
                          'launched_by_bench': os.environ.get('SB_BENCH_LAUNCHED') == '1'}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    launched = 'RANK' in os.environ or 'LOCAL_RANK' in os.environ
    if args.gpus > 1 and not launched:
        sys.exit(self_launch(args))
    if args.dry_run:
        return dry_run(args)
    if args.realistic:
        return run_realistic(args)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world > 1 or args.gpus > 1 or os.environ.get('SB_FORCE_DIST') == '1':   # (diagnostic: sharded path at N=1)
        if args.heuristic is None:
            args.heuristic = 'efficiency'   # C5
        import bench_dist
        return bench_dist.main(args)
    if args.heuristic is None:
        args.heuristic = 'balanced'         # C3
    per, elapsed, el_eng, segs, (first, length, turns, engines), vsum = run_single(args)
    parents = sum(p['n_parents'] for p in per)
    raw = sum(p['n_raw'] for p in per)
    uniq = sum(p['n_unique'] for p in per)
    kept = sum(p['n_kept'] for p in per)
    phases = {k: round(sum(p[k] for p in per) / len(per), 3) for k in
              ('ms_expand', 'ms_survive', 'ms_mt', 'ms_emit', 'ms_select', 'ms_gather', 'ms_total')}
    dom = max(('ms_expand', 'ms_survive', 'ms_emit', 'ms_select', 'ms_gather'), key=lambda k: phases[k])
    # roofline of the dominant phase (k_expand in practice): the contract's algorithmic bytes — SURVEY §8(d)'s
    # 28 + 20 b_raw + 37 b_uniq + 33 per parent, times the parents one launch expands — over its device time
    # (VERDICT r4 item 5); the expansion-only byte model (what k_expand itself reads and writes) rides beside it
    ms_dom = phases[dom]
    n_par = parents / len(per)
    byt = step_bytes(n_par, raw / len(per), uniq / len(per), kept / len(per))
    achieved = byt / (ms_dom * 1e-3) / 1e9 if ms_dom > 0 else 0.0
    xbyt = expand_bytes(n_par, raw / len(per), uniq / len(per))
    x_ach = xbyt / (ms_dom * 1e-3) / 1e9 if ms_dom > 0 else 0.0
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
        'data': f'synthetic: seeded solve trajectory (random.seed({args.seed})); timed: the saturated turns '
                f'{first}..{first + length - 1} of the {turns}-move goal-{GOAL} solve (queue full, no goal state), '
                f'replayed on {engines} seeded engines set up outside the timed region',
        'config': {'workload': f'speedrun goal_pts={GOAL} -u -H {args.heuristic} beam_width={args.width} (C3)',
                   'beam_width': args.width, 'heuristic': args.heuristic, 'seed': args.seed,
                   'parallelism': 'single GPU', 'b_raw': round(raw / parents, 3), 'b_uniq': round(uniq / parents, 3),
                   'timed_turns': [first, first + length - 1], 'moves': turns,
                   'timed_expansions': ('engine lookahead at the window edges: the turn after each segment'
                                        if args.lookahead_edges else 'exactly the timed turns\' own'),
                   'segment_end': ('the engine stream (legacy: noise generated for later turns not waited for)'
                                   if args.engine_stream_end else 'every stream (noise generated in the segment charged to it)'),
                   'segments': segs, 'warmup_engine': 'own (the timed steps start on fresh engines)',
                   'visited': vsum},
        'value_engine_stream_end': round(parents / el_eng, 1),
        'phases_ms': phases,
        'roofline': {'bound': 'hbm', 'kernel': dom.replace('ms_', 'k_'), 'achieved': round(achieved, 2),
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 5),
                     'algorithmic_bytes_per_launch': int(byt),
                     'byte_model': 'SURVEY §8(d): 28 + 20 b_raw + 37 b_uniq + 33 B per parent, x the launch\'s parents',
                     'launch_ms': ms_dom, 'traffic': None,
                     'frac_expand_model': round(x_ach / HBM_PEAK_GBS, 5), 'expand_model_bytes_per_launch': int(xbyt)},
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
        # round 4: the same launch priced at the two rates calibrated with the counters on a 32 GiB table
        # (profiles/micro/fetchcal.hip): a probe that settles with its load, and an insert (probe + tag CAS + key
        # store on one line); displacing claims (atomicMin + lost mark) are left out, so this is a lower bound
        new = uniq / len(per)
        t_bound = ((raw / len(per) - new) / RANDOM_PROBE_G + new / RANDOM_INSERT_G) / 1e9 * 1e3
        out['roofline']['random_access'].update({
            'calibrated_bound_ms': round(t_bound, 3), 'frac_calibrated': round(t_bound / ms_dom, 3),
            'calibrated_rates_G_per_s': {'probe': RANDOM_PROBE_G, 'insert': RANDOM_INSERT_G},
            'calibration_source': 'profiles/r4/s2/fetchcal_plain.txt, fetchcal_pmc.txt (FETCH_SIZE x2 = 128 B per '
                                  'random 16-B probe, the guide\'s gfx950 correction holds for random lines too)'})
    tr, tns, hit, src = pmc_traffic(dom.replace('ms_', 'k_'))
    if tr is not None:
        out['roofline']['traffic'] = int(tr)
        out['roofline']['traffic_GBps'] = round(tr / (tns * 1e-9) / 1e9, 1)
        if hit is not None:
            out['roofline']['l2_hit_rate'] = round(hit, 4)
        out['roofline']['traffic_source'] = f'{src} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; ' \
                                            f'hbm = (2*FETCH + WRITE) KiB, gfx950 correction)'
    if not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(args.width, args.heuristic, args.seed, first)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
