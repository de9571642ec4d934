#!/bin/bash
# Round 6, session 13: the 8-part world-1 key-pass run that once took 286 ms per step (r6s12 p8_2): repeated under
# kernel traces to see which kernel, if it recurs
O=${1:-gpurun_out/r6s13}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4; do
    SB_DIST_PARTS=8 SB_FORCE_DIST=1 SB_DIST_KP1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_p8_$i -o run -- \
        python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/kp1_p8_$i.json 2> $O/kp1_p8_$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/kp1_p8_$i.json')); print('kp1 p8 $i', round(d['value']/1e6,1), d['ms_per_step'])"
    python3 - <<PY
import csv
rows = sorted(csv.DictReader(open('$O/tr_p8_$i/run_kernel_stats.csv')), key=lambda r: -float(r['MaxNs']))[:4]
for r in rows: print('   max', r['Name'][:50], round(float(r['MaxNs']) / 1e6, 3), 'ms, avg', round(float(r['AverageNs']) / 1e6, 3))
PY
    rm -f $O/tr_p8_$i/run_kernel_trace.csv
done
