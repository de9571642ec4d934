"""Command line, flag-compatible with the reference's splendor_fastest_win.py:14-152.

Same flags and output; adds --seed (random.seed before the solve, and the realistic market shuffle
seed, for reproducible runs), --device (GPU ordinal) and --gpus N (the speedrun beam sharded over N GPUs,
one worker process each: splendor_amd.multi).  The solve runs on the MI355X engine.
"""
from __future__ import annotations

import argparse
import random
import sys

from .buys import export_buys_to_txt, load_buys
from .deck import Color
from .realistic import GameConfig, MultiPlayerState
from .solver import HEURISTICS, State
from .ui import render_solution


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description='A tool to bruteforce fastest winning moves for the board game Splendor.')
    p.add_argument('goal_pts', help='target amount of points', nargs='?', type=int)
    p.add_argument('-u', '--use_heuristic', help='use a heuristic formula to limit the search space of BFS',
                   action='store_true')
    p.add_argument('-b', '--buys', help='regenerate and store all possible buys', action='store_true')
    p.add_argument('-e', '--export', help='export possible buys to a .txt file', action='store_true')
    p.add_argument('-r', '--render', help='render the solution with the UI', action='store_true')
    p.add_argument('-H', '--heuristic', help=f'heuristic function to use (choices: {", ".join(HEURISTICS.keys())})',
                   default='simple', choices=list(HEURISTICS.keys()))
    p.add_argument('-w', '--beam_width', help='maximum states to keep per turn when using heuristic (default: 300000)',
                   type=int, default=300_000)
    p.add_argument('-q', '--quiet', help='suppress progress output during solving', action='store_true')
    p.add_argument('--realistic', help='use realistic 2-player mode with gem pool and card visibility constraints',
                   action='store_true')
    p.add_argument('--players', help='number of players for realistic mode (default: 2)', type=int, default=2)
    p.add_argument('--shuffle', help='shuffle card market in realistic mode', action='store_true')
    p.add_argument('--seed', help='seed random (and the realistic market shuffle) for a reproducible run',
                   type=int, default=None)
    p.add_argument('--device', help='GPU ordinal (default 0)', type=int, default=0)
    p.add_argument('--gpus', help='shard the speedrun beam over N GPUs, one process each (default 1); RCCL between '
                                  'the GPUs (its asynchronous exchanges are verified with a completion-contract test '
                                  'double and gloo, not yet on a multi-GPU node: SB_DIST_BACKEND=gloo forces gloo).  The trail '
                                  'is owned by key hash, bit-exact; SB_DIST_MIG=1 (card-set ownership, faster) is NOT '
                                  'bit-exact by construction: two card sets with an equal 64-bit key are both kept',
                   type=int,
                   default=1)
    return p


def cli(argv=None):
    parser = build_parser()
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) == 0:
        parser.print_help()
        parser.exit()
    args = parser.parse_args(argv)
    if args.gpus < 1:
        parser.error('--gpus must be >= 1')
    if args.gpus > 1 and args.realistic:
        parser.error('--gpus > 1 shards the speedrun solve; --realistic runs on one GPU')
    if args.seed is not None:
        random.seed(args.seed)
    try:
        if args.export:
            export_buys_to_txt()
            return
        if args.buys:
            load_buys(update=True)
        if args.goal_pts:
            if args.realistic:
                gems_per_color = {2: 4, 3: 5, 4: 7}.get(args.players, 4)
                config = GameConfig(num_players=args.players, target_points=args.goal_pts,
                                    gems_per_color=gems_per_color, infinite_resources=False)
                root = MultiPlayerState.newgame(config=config, shuffle_market=args.shuffle,
                                                seed=args.seed if args.shuffle else None)
                if args.seed is not None:
                    random.seed(args.seed)
                solution = root.solve(use_heuristic=True, heuristic_name='competitive',
                                      beam_width=args.beam_width if args.beam_width != 300_000 else 20_000,
                                      verbose=not args.quiet, device=args.device)
                if solution:
                    last = solution[-1]
                    print(f'\n{"=" * 60}')
                    print(f'Game Over! Winner: Player {last.get_winner()}')
                    print('Final Scores:')
                    for p in last.players:
                        print(f'  Player {p.player_id}: {p.pts} points, {len(p.cards)} cards')
                    print(f'Total moves: {last.turn_number}')
                    print(f'{"=" * 60}\n')
                    if args.render:
                        print('Move-by-move breakdown:')
                        for i, state in enumerate(solution):
                            print(f'\nMove {i}: {state}')
                            for p in state.players:
                                print(f'  P{p.player_id}: {p.pts}pts, gems={p.gems}, bonus={p.bonus}')
            else:
                solution = State.newgame().solve(goal_pts=args.goal_pts, use_heuristic=args.use_heuristic,
                                                 heuristic_name=args.heuristic, beam_width=args.beam_width,
                                                 verbose=not args.quiet, device=args.device, gpus=args.gpus)
                if args.render:
                    render_solution(solution)
                else:
                    print('\nSolution:')
                    print(f'({", ".join(c.name.title() for c in Color)}) Cards')
                    for state in solution:
                        print(state)
    except KeyboardInterrupt:
        print('Execution stopped by the user.')
        parser.exit()


if __name__ == '__main__':
    cli()
