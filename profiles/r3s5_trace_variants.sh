#!/bin/bash
# round 3, session 5: rocprofv3 kernel trace of C3 (6 timed steps) for each variant library in
# splendor_amd/variants/, summarised per kernel.  Usage (repo root): bash profiles/r3s5_trace_variants.sh OUTDIR
O=${1:-gpurun_out/s5v}; mkdir -p $O
export TMPDIR=/tmp
for f in splendor-rl-gym_amd/splendor_amd/variants/*.so; do
  v=$(basename $f .so)
  SPLENDOR_BEAM_LIB=$PWD/$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
      python3 bench.py --no-cpu-baseline --steps 6 --warmup 0 > $O/$v.json 2> $O/$v.err || exit $?
  python3 profiles/summarize.py $O/$v --steps 6 --out $O/$v.summary.json > /dev/null 2>&1
  python3 - $O/$v <<'PY'
import csv, glob, sys, collections, re
d = sys.argv[1]
f = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
ex = [i for i, r in enumerate(rows) if r['Kernel_Name'].split('(')[0].endswith('k_expand<false>') or 'k_expand<false>' in r['Kernel_Name']]
start = ex[-6]
agg = collections.defaultdict(lambda: [0, 0])
for r in rows[start:]:
    n = re.sub(r'^(void )?(sb::)?', '', r['Kernel_Name']).split('(')[0]
    agg[n][0] += 1
    agg[n][1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
print(d)
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f'  {n:40s} {c:4d} {t / 6 / 1e3:9.1f} us/step')
PY
done
