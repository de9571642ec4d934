#!/bin/bash
# FETCH_SIZE calibration passes (one counter group per rocprofv3 run) for profiles/micro/fetchcal.hip
O=${1:-gpurun_out/fetchcal}; mkdir -p $O
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result -o $O/fetchcal profiles/micro/fetchcal.hip || exit $?
timeout -k 10 120 $O/fetchcal 32 100 > $O/plain.txt 2>&1 || exit $?
cat $O/plain.txt
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc $pmc --output-format csv -d $O/p$i -o run -- $O/fetchcal 32 100 > $O/p$i.txt 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i ($pmc) failed: $rc"; [ $rc -ge 124 ] && exit $rc; fi
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, 'p*', '**', '*counter_collection.csv'), recursive=True)):
    agg = {}
    for r in csv.DictReader(open(f)):
        k = (r['Kernel_Name'].split('(')[0], r['Counter_Name'])
        agg[k] = agg.get(k, 0.0) + float(r['Counter_Value'])
    for (kn, cn), v in sorted(agg.items()):
        print(f'{kn:12s} {cn:24s} {v:16.0f}')
PY
