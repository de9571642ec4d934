"""bench.py --gpus N without a launcher starts torch.distributed.run itself (one process per GPU): the
plumbing is checked on CPU with --dry-run (gloo group, no GPU call) — rank 0 reports the world size."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*argv):
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE')}
    p = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), *argv], capture_output=True, text=True,
                       timeout=240, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_self_launch_world_2():
    out = _run('--gpus', '2', '--dry-run')
    assert out['n_gpus'] == 2 and out['launched_by_bench']


def test_single_process_world_1():
    out = _run('--gpus', '1', '--dry-run')
    assert out['n_gpus'] == 1 and not out['launched_by_bench']
