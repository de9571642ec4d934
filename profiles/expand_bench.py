"""Device time of the expansion's variants on C3's saturated queue (sb_debug_expand_bench): the single-GPU
fused k_expand, the sharded expansion at world 1 / world 8 / owning nothing (the key pass alone), the owner
claims of every record, and the key pass beside the claims on two streams (can they overlap?).
    python3 profiles/expand_bench.py [--turn 11] [--reps 3] [--width 4000000] [--heuristic balanced]"""
import argparse
import ctypes as C
import json
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'splendor-rl-gym_amd'))
from splendor_amd import _lib as L   # noqa: E402
from splendor_amd.engine import HEURISTIC_IDS, BeamEngine   # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--turn', type=int, default=11)
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--width', type=int, default=4_000_000)
ap.add_argument('--heuristic', default='balanced')
a = ap.parse_args()
random.seed(0)
eng = BeamEngine(goal_pts=15, use_heuristic=True, heuristic=HEURISTIC_IDS[a.heuristic], beam_width=a.width,
                 mt_state625=random.getstate()[1], device=0)
for t in range(a.turn):
    if t == a.turn - 1:
        eng.set_lookahead(False)
    st = eng.step()
    print(f'turn {t}: parents {st["n_parents"]} unique {st["n_unique"]} kept {st["n_kept"]}', file=sys.stderr, flush=True)
lib = L.lib()
lib.sb_debug_expand_bench.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
out = (C.c_float * 20)()
L.check(lib.sb_debug_expand_bench(eng._h, a.reps, out), 'sb_debug_expand_bench')
names = ['expand_fused_1gpu', 'sharded_w1', 'sharded_w8_rank0', 'sharded_w8_no_own', 'claims_all_records',
         'no_own_beside_claims_wall', 'raw_count_scan', 'raw_children', 'keypass_a_w8', 'keypass_scan_b_w8',
         'dbg_a_no_claims', 'dbg_a_no_claims_cheap_key', 'dbg_a_no_claims_key_stores', 'dbg_a_no_claims_no_stores',
         'keys_a_no_own_beside_claims_wall', 'keys_a_no_own', 'pipelined_dedup_w8_two_streams',
         'pipelined_dedup_w8_one_stream', 'pipelined_dedup_w8_priority_streams', 'stream_priority_levels']
res = {k: round(float(v), 4) for k, v in zip(names, out)}
res.update(turn=a.turn, parents=eng.turn_size(a.turn), width=a.width, heuristic=a.heuristic, reps=a.reps)
print(json.dumps(res), flush=True)
