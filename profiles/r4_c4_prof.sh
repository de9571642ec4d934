#!/bin/bash
# Round 4: C4 kernel trace + PMC passes (collect_r3_c4.sh) of the k_rexpand2 build, summarised
O=${1:-gpurun_out/r4c4p}
bash profiles/collect_r3_c4.sh $O || exit $?
python3 profiles/summarize.py $O --expand k_rexpand2 --steps 6 --out $O/r4_c4_profile_summary.json | tail -25
