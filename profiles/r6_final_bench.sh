#!/bin/bash
# Round 6, final tree: the driver's default bench line (N=1, with cpu_baseline), the C3 kernel trace + PMC passes
# (collect_r3.sh) summarised into r6_profile_summary.json, the C4 line, the KP1 line
O=${1:-gpurun_out/r6finalb}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; cat $O/bench_n1.json; [ $rc -eq 0 ] || exit $rc
bash profiles/collect_r3.sh $O/prof || exit $?
python3 profiles/summarize.py $O/prof --steps 6 --out $O/prof/r6_profile_summary.json | tail -12
timeout -k 10 300 python3 bench.py --realistic --steps 12 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
rc=$?; python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('C4', round(d['value']/1e6,1), d['ms_per_step'])"; [ $rc -eq 0 ] || exit $rc
SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1.json 2> $O/kp1.err
rc=$?; python3 -c "import json; d=json.load(open('$O/kp1.json')); print('KP1', round(d['value']/1e6,1), d['ms_per_step'])"; exit $rc
