#!/usr/bin/env python3
"""Build tuning variants of libsplendor_beam.so (same sources, -D knobs of sb_engine.hip) into
splendor-rl-gym_amd/splendor_amd/variants/, and bench each on the GPU box:
    python profiles/variants.py build NAME=DEF1,DEF2 ...     (here, cross-compiling for gfx950)
    python profiles/variants.py bench [--steps K]             (GPU box: SPLENDOR_BEAM_LIB=... bench.py)
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'splendor-rl-gym_amd'))
VDIR = os.path.join(REPO, 'splendor-rl-gym_amd', 'splendor_amd', 'variants')


def main():
    if sys.argv[1] == 'build':
        from concurrent.futures import ThreadPoolExecutor

        from splendor_amd import _lib
        os.makedirs(VDIR, exist_ok=True)
        jobs = []
        for spec in sys.argv[2:]:
            name, _, defs = spec.partition('=')
            jobs.append((os.path.join(VDIR, f'lib_{name}.so'), tuple(d for d in defs.split(',') if d)))
        with ThreadPoolExecutor(4) as ex:
            for out in ex.map(lambda j: _lib.build(out=j[0], defines=j[1]), jobs):
                print('built', out)
    else:
        steps = sys.argv[sys.argv.index('--steps') + 1] if '--steps' in sys.argv else '8'
        modes = ['single', 'sharded'] if '--dist' in sys.argv else ['single']   # sharded: SB_FORCE_DIST=1 (N=1)
        for f in sorted(os.listdir(VDIR)):
            for mode in modes:
                env = dict(os.environ, SPLENDOR_BEAM_LIB=os.path.join(VDIR, f))
                if mode == 'sharded':
                    env['SB_FORCE_DIST'] = '1'
                extra = ['--realistic'] if '--realistic' in sys.argv else []   # config C4 instead of C3
                r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--no-cpu-baseline', '--steps',
                                    steps] + extra, env=env, capture_output=True, text=True, timeout=300)
                line = [l for l in r.stdout.splitlines() if l.startswith('{')]
                if not line:
                    print(f, mode, 'FAILED', r.stderr[-500:], flush=True)
                    continue
                d = json.loads(line[0])
                print(f'{f:28s} {mode:8s} {d["value"] / 1e6:8.1f} M/s  {d["ms_per_step"]:.3f} ms  '
                      f'{d.get("phases_ms", "")}', flush=True)


if __name__ == '__main__':
    main()
