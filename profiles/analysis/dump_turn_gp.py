import random, sys
import numpy as np
sys.path[:0] = ['/root/repo/oracle', '/root/repo/splendor-rl-gym_amd']
import oracle_c
from splendor_amd.deck import deck_rows
width, turn, heur = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
random.seed(0)
o = oracle_c.OracleSolve(15, use_heuristic=True, heuristic_name=heur, beam_width=width, mt_state625=random.getstate()[1])
for t in range(turn):
    o.step()
lo, hi, par, _ = o.turn_arrays(turn)
with open(f'/tmp/gp_w{width}_t{turn}.bin', 'wb') as f:
    f.write(np.array([len(lo)], dtype=np.int64).tobytes())
    f.write(lo.astype(np.uint64).tobytes()); f.write(hi.astype(np.uint64).tobytes()); f.write(par.astype(np.uint32).tobytes())
np.array(deck_rows(), dtype=np.int32).tofile('/tmp/deck.bin')
print(len(lo), par[:10])
