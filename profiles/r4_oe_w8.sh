#!/bin/bash
# Round 4: serialised world-8 traces (C5 shape, 4M per rank, visited 2^29 per rank) of the card-set protocol with
# owner emission (flags 800) and without (288), same box, each with its phase table and projection
O=${1:-gpurun_out/r4oew}; mkdir -p $O
for v in oe:800 mig:288; do
  name=${v%%:*}; fl=${v##*:}
  bash profiles/collect_r4_mig.sh $O/$name 8 29 5 $fl || exit $?
  python3 profiles/sharded_table.py $O/$name --world 8 --steps 5 --out $O/${name}_table.json | grep -v "^rank" | tail -19
  python3 profiles/project_n8.py $O/${name}_table.json $O/$name/bench_r0.json --single-ms 4.507 | grep -v "^{"
done
