#!/bin/bash
# Round 4: serialised world-8 traces (C5 shape, 4M per rank, visited 2^29 slots per rank as round 3's table) of
# both sharded protocols on one box — card-set ownership (flags 288) and key ownership (flags 32) — each
# with its phase table; then C4's claim statistics + the FETCH_SIZE calibration (r4_c4_attrib.sh)
O=${1:-gpurun_out/r4w}; mkdir -p $O
bash profiles/collect_r4_mig.sh $O/mig 8 29 5 288 || exit $?
python3 profiles/sharded_table.py $O/mig --world 8 --steps 5 --out $O/mig_table.json | tail -18
bash profiles/collect_r3_sharded.sh $O/key 8 29 5 || exit $?
python3 profiles/sharded_table.py $O/key --world 8 --steps 5 --out $O/key_table.json | tail -18
bash profiles/r4_c4_attrib.sh $O/c4 || exit $?
