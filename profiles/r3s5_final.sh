#!/bin/bash
# round 3, session 5 end: full -m gpu suite, smoke, the driver's bench command, sharded N=1, C4 (round_end.sh),
# then the C3 kernel profile of the final build (trace + FETCH/WRITE/TCC passes) and its summary
O=${1:-gpurun_out/s5z}
bash profiles/round_end.sh $O || exit $?
bash profiles/collect_r3.sh $O/prof || exit $?
python3 profiles/summarize.py $O/prof --steps 6 --out $O/r3s5_profile_summary.json > $O/summarize.txt 2>&1 || exit $?
tail -16 $O/summarize.txt
