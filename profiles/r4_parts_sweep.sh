mkdir -p gpurun_out/k11
for P in 1 2 4 8; do SB_BENCH_PARTS=$P timeout -k 10 200 python3 profiles/expand_bench.py --turn 11 --reps 2 > gpurun_out/k11/p$P.json 2>/dev/null || exit 1; done
for G in 1024 4096; do SB_BENCH_CLAIM_GRID=$G timeout -k 10 200 python3 profiles/expand_bench.py --turn 11 --reps 2 > gpurun_out/k11/g$G.json 2>/dev/null || exit 1; done
for f in gpurun_out/k11/*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print({k: d[k] for k in ('claims_all_records','keypass_a_w8','pipelined_dedup_w8_two_streams','pipelined_dedup_w8_one_stream','pipelined_dedup_w8_priority_streams')})"; done
