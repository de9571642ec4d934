#!/bin/bash
# round 4: serialised world-8 traces of the card-set protocol (C5 shape, 4M per rank) + phase table + N=8
# projection; then the world-2 PMC passes of its key kernel
O=${1:-gpurun_out/r4p}; mkdir -p $O
bash profiles/collect_r4_mig.sh $O/w8 8 28 5 288 || exit $?
python3 profiles/sharded_table.py $O/w8 --world 8 --steps 5 --out $O/w8_table.json | tail -20
python3 profiles/project_n8.py $O/w8_table.json $O/w8/bench_r0.json > $O/projection.txt 2>&1; cat $O/projection.txt | head -8
bash profiles/collect_r4_mig_pmc.sh $O/pmc 257 4 || exit $?
python3 profiles/pmc_sharded.py $O/pmc --kernel k_mkeys_a --steps 4 --out $O/r4_mig_w2_pmc.json
