"""Dump a saturated turn's parents (C3 trajectory by default) for profiles/analysis/dupstats.c."""
import random
import sys

import numpy as np

sys.path[:0] = ['oracle', 'splendor-rl-gym_amd']
import oracle_c  # noqa: E402
from splendor_amd.deck import deck_rows  # noqa: E402

width, turn, heur = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
random.seed(0)
o = oracle_c.OracleSolve(15, use_heuristic=True, heuristic_name=heur, beam_width=width, mt_state625=random.getstate()[1])
for t in range(turn):
    o.step()
lo, hi, _, _ = o.turn_arrays(turn)
with open(f'/tmp/parents_w{width}_t{turn}.bin', 'wb') as f:
    f.write(lo.tobytes())
    f.write(hi.tobytes())
np.array(deck_rows(), dtype=np.int32).tofile('/tmp/deck.bin')
print(len(lo))
