#!/bin/bash
# Round 6, session 16: C4's k_rexpand2 at 6 and 7 waves per SIMD (80 / 72 VGPRs, spills) against the default 5 (96 VGPRs),
# interleaved three times
O=${1:-gpurun_out/r6s16}; mkdir -p $O
export TMPDIR=/tmp
c4() {   # name, lib
    SPLENDOR_BEAM_LIB=$2 timeout -k 10 200 python3 bench.py --realistic --no-cpu-baseline --steps 12 --warmup 2 > $O/c4_$1.json 2> $O/c4_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/c4_$1.json')); print('$1', round(d['value']/1e6,1), d['ms_per_step'], d.get('phases_ms'))"
}
D=splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so
c4 w5_1 $D && c4 w6_1 ab/libsb_rx6.so && c4 w7_1 ab/libsb_rx7.so && c4 w5_2 $D && c4 w6_2 ab/libsb_rx6.so && c4 w7_2 ab/libsb_rx7.so && c4 w5_3 $D && c4 w6_3 ab/libsb_rx6.so && c4 w7_3 ab/libsb_rx7.so
