#!/bin/bash
# Round 4: where C4's k_rexpand traffic comes from.  (1) the claim-statistics build
# (SB_CLAIM_STATS: per turn, keys found from earlier turns / inserted / same-turn early-outs / lost at the
# atomicMin / displacing claims) on the C4 bench window, (2) the per-operation HBM bytes of the same access
# kinds from profiles/micro/fetchcal.hip (FETCH_SIZE / WRITE_SIZE per random probe, CAS, store, atomicMin).
# The stats variant is built here (python profiles/variants.py build stats=SB_CLAIM_STATS) and shipped.
O=${1:-gpurun_out/r4c4}; mkdir -p $O
V=splendor-rl-gym_amd/splendor_amd/variants/lib_stats.so
SPLENDOR_BEAM_LIB=$V timeout -k 10 300 python3 -u bench.py --realistic --no-cpu-baseline --steps 6 --warmup 0 \
    > $O/bench_c4_stats.json 2> $O/bench_c4_stats.err || exit $?
grep rclaims $O/bench_c4_stats.err | tail -12
bash profiles/micro/fetchcal.sh $O/fetchcal || exit $?
