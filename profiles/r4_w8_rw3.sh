#!/bin/bash
# Round 4: serialised world-8 traces after the 3-word kept records (key ownership, flags 32, and card-set
# ownership without owner emission, flags 288): phase tables + N=8 projections
O=${1:-gpurun_out/r4w3}; mkdir -p $O
bash profiles/collect_r3_sharded.sh $O/key 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/key --world 8 --steps 5 --out $O/key_table.json | grep -v "^rank" | tail -19
python3 profiles/project_n8.py $O/key_table.json $O/key/bench_r0.json --single-ms 4.507 | grep -v "^{"
bash profiles/collect_r4_mig.sh $O/mig 8 29 5 288 || exit $?
python3 profiles/sharded_table.py $O/mig --world 8 --steps 5 --out $O/mig_table.json | grep -v "^rank" | tail -19
python3 profiles/project_n8.py $O/mig_table.json $O/mig/bench_r0.json --single-ms 4.507 | grep -v "^{"
