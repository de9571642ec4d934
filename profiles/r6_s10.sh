#!/bin/bash
# Round 6, session 10: C3 select A/B of the LSD sort passes — scattered writes replaced by coalesced ones (SB_OS_DBG=2,
# timing only: wrong order) and a 12-predecessor look-back window, interleaved with the default build
O=${1:-gpurun_out/r6s10}; mkdir -p $O
export TMPDIR=/tmp
c3() {   # name, lib
    SPLENDOR_BEAM_LIB=$2 timeout -k 10 200 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/c3_$1.json 2> $O/c3_$1.err || return 1
    python3 -c "import json; d=json.load(open('$O/c3_$1.json')); print('$1', round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"
}
D=splendor-rl-gym_amd/splendor_amd/libsplendor_beam.so
c3 base1 $D && c3 dbg2_1 ab/libsb_osdbg2.so && c3 lb12_1 ab/libsb_oslb12.so && c3 base2 $D && c3 dbg2_2 ab/libsb_osdbg2.so && c3 lb12_2 ab/libsb_oslb12.so
