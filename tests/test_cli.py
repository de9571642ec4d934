"""CLI mirror of splendor_fastest_win.py (flags, buys exports, output format), and the UI renderer."""
import os
import subprocess
import sys

import pytest

from conftest import REPO, golden
from splendor_amd import buys as B
from splendor_amd import ui
from splendor_amd.cli import build_parser
from splendor_amd.solver import State

SCRIPT = os.path.join(REPO, 'splendor-rl-gym_amd', 'splendor_fastest_win.py')


def test_flags_match_reference():
    a = build_parser().parse_args(['15', '-u', '-H', 'balanced', '-w', '1000', '-q', '-r'])
    assert (a.goal_pts, a.use_heuristic, a.heuristic, a.beam_width, a.quiet, a.render) == (15, True, 'balanced', 1000,
                                                                                          True, True)
    a = build_parser().parse_args(['15', '--realistic', '--players', '3', '--shuffle'])
    assert a.realistic and a.players == 3 and a.shuffle and a.beam_width == 300_000
    assert build_parser().parse_args([]).goal_pts is None
    with pytest.raises(SystemExit):
        build_parser().parse_args(['3', '-H', 'nope'])


def test_no_arguments_prints_help():
    out = subprocess.run([sys.executable, SCRIPT], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and 'usage:' in out.stdout and '--beam_width' in out.stdout


def test_possible_buys_matches_reference_table():
    b = B.possible_buys()
    assert len(b) == 8 ** 5
    for g, exp in golden('tables.json')['buys_sample']:
        assert list(b[tuple(g)]) == exp


def test_export_and_store(tmp_path):
    B.export_buys_to_txt(tmp_path / 'buys.txt')
    lines = (tmp_path / 'buys.txt').read_text().splitlines()
    assert len(lines) == 8 ** 5 and lines[0].startswith('(0, 0, 0, 0, 0): ()')
    b = B.load_buys(update=True, path=tmp_path / 'buys.pickle')
    assert B.load_buys(path=tmp_path / 'buys.pickle') == b


def test_render_solution_format(capsys):
    s0 = State.newgame()
    s1 = State((), (0,) * 5, (1, 1, 0, 0, 1), 0, 0).buy_card(0)
    ui.render_solution([s0, s1])
    out = capsys.readouterr().out
    assert 'SOLUTION PATH' in out and '=== Step 0 ===' in out and 'Held Gems: None' in out
    assert '=== Step 1 ===' in out and 'Cards: ' + str(ui.deck[0]) in out
    assert f'FINAL: {s1.pts} points in 1 moves' in out
    assert ui.format_gems((2, 0, 1, 0, 0)) == 'White: 2, Green: 1'
    assert ui.format_cards(()) == 'None'


@pytest.mark.gpu
def test_cli_speedrun_on_gpu():
    """`6 -u -w 1000 --seed 0` prints the reference's solution (solves_small[0], captured from the reference)."""
    g = golden('solves_small.json')[0]
    assert (g['goal'], g['heuristic'], g['beam_width'], g['seed']) == (6, 'simple', 1000, 0)
    out = subprocess.run([sys.executable, SCRIPT, '6', '-u', '-w', '1000', '-q', '--seed', '0'],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    body = out.stdout.split('\nSolution:\n', 1)[1].splitlines()
    assert body[0] == '(White, Blue, Green, Red, Black) Cards'
    assert body[1:1 + len(g['path'])] == [p[4] for p in g['path']]


@pytest.mark.gpu
def test_cli_realistic_on_gpu():
    """`6 --realistic -w 3000 --seed 0` reaches the reference's game over (realistic_g6_p2_fixed_w3000_s0)."""
    g = golden('realistic_g6_p2_fixed_w3000_s0.json')
    out = subprocess.run([sys.executable, SCRIPT, '6', '--realistic', '-w', '3000', '-q', '--seed', '0', '-r'],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert f'Game Over! Winner: Player {g["winner"]}' in out.stdout
    assert f'Total moves: {g["moves"]}' in out.stdout
    for pid, cards, _gems, _bonus, pts, _saved in g['final']:
        assert f'  Player {pid}: {pts} points, {len(cards)} cards' in out.stdout
    assert 'Move-by-move breakdown:' in out.stdout and f'Move {g["moves"]}: ' in out.stdout


# the reference's lazy buys-table loader prints these on its first get_buys() (src/buys.py:25-36); the engine
# tests affordability on the device and loads no table, so they are the one difference in the stdout
_BUYS_MESSAGES = {'Unpickling buys...', 'Generating buys...', 'Pickling buys...', 'Pickling finished.'}


@pytest.mark.gpu
@pytest.mark.parametrize('case', range(5))
def test_cli_verbose_output_matches_reference(case):
    """Full stdout without -q (banner, turn= / max_pts= progress lines, realistic every-100-turns line, solution
    or render) equals the reference CLI's under random.seed(0) (tests/golden/cli_verbose.json)."""
    g = golden('cli_verbose.json')[case]
    out = subprocess.run([sys.executable, SCRIPT, *g['argv'], '--seed', str(g['seed'])], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    exp = [ln for ln in g['stdout'].splitlines() if ln not in _BUYS_MESSAGES]
    assert out.stdout.splitlines() == exp


def test_gpus_flag():
    a = build_parser().parse_args(['15', '-u', '--gpus', '4'])
    assert a.gpus == 4 and build_parser().parse_args(['15']).gpus == 1
    for bad in (['15', '--gpus', '0'], ['15', '--realistic', '--gpus', '2']):
        out = subprocess.run([sys.executable, SCRIPT, *bad], capture_output=True, text=True, timeout=120)
        assert out.returncode == 2 and '--gpus' in out.stderr


def test_multi_gpu_launcher_dry_run():
    """State.solve(gpus=N) / --gpus N start N worker processes with torch.distributed.run (never touching
    the GPU in the caller); the plumbing on CPU: the workers join one gloo world, rank 0 reports back."""
    from splendor_amd.multi import launch
    assert launch({'dry_run': True}, 2) == {'dry_run': True, 'world': 2}


@pytest.mark.gpu
@pytest.mark.parametrize('argv', [['8', '-u', '-H', 'efficiency', '-w', '20000', '--seed', '0'],
                                  ['10', '-u', '-H', 'balanced', '-w', '3000', '--seed', '0']])
def test_cli_gpus_2_matches_one_gpu(argv):
    """`--gpus 2` (2 ranks on one GPU, gloo transport) prints exactly what the single-GPU run prints:
    banner, every turn= / max_pts= line, the solution."""
    env = dict(os.environ, SB_DIST_BACKEND='gloo')
    one = subprocess.run([sys.executable, SCRIPT, *argv], capture_output=True, text=True, timeout=300, env=env)
    two = subprocess.run([sys.executable, SCRIPT, *argv, '--gpus', '2'], capture_output=True, text=True, timeout=300,
                         env=env)
    assert one.returncode == 0, one.stderr[-2000:]
    assert two.returncode == 0, two.stderr[-2000:]
    assert '\nSolution:\n' in one.stdout and 'max_pts=' in one.stdout
    assert two.stdout == one.stdout
