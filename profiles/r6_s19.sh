#!/bin/bash
# Round 6, session 19: where the key pass's time goes — the expansion micro-bench (sb_debug_expand_bench) on C3's
# turn 11 queue with the default build and with SB_KS_SPLIT=1: the key pass with real keys, a stand-in key (no
# hashing) and no stores
O=${1:-gpurun_out/r6s19}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python3 profiles/expand_bench.py --turn 11 --reps 3 > $O/eb_default.json 2> $O/eb_default.err || exit 1
SPLENDOR_BEAM_LIB=ab/libsb_split.so timeout -k 10 240 python3 profiles/expand_bench.py --turn 11 --reps 3 > $O/eb_split.json 2> $O/eb_split.err || exit 1
for f in default split; do python3 -c "
import json; d=json.load(open('$O/eb_$f.json'))
print('$f', {k: d[k] for k in ('keypass_a_w8','keypass_scan_b_w8','dbg_a_no_claims','dbg_a_no_claims_cheap_key','dbg_a_no_claims_key_stores','dbg_a_no_claims_no_stores','keys_a_no_own','expand_fused_1gpu')})"; done
