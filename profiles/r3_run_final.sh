#!/bin/bash
# round 3 end: full -m gpu suite, smoke, the driver's bench command, sharded N=1, C4, then the C3 profile
O=${1:-gpurun_out/r3k}
bash profiles/round_end.sh $O || exit $?
bash profiles/collect_r3.sh $O/prof || exit $?
python3 profiles/summarize.py $O/prof --steps 6 --out $O/r3_profile_summary.json
