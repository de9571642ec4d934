#!/bin/bash
# Round 4: C3 kernel trace + PMC passes of this round's build (collect_r3.sh), summarised
O=${1:-gpurun_out/r4c3p}
bash profiles/collect_r3.sh $O || exit $?
python3 profiles/summarize.py $O --steps 6 --out $O/r4_profile_summary.json | tail -20
