set -e
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_custom.py tests/test_gpu_engine.py tests/test_gpu_realistic.py tests/test_gpu_big.py -k "not c5" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python3 -u bench.py --realistic --steps 12 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
tail -1 $O/bench_c4.json
timeout -k 10 300 python3 -u bench.py --realistic --steps 12 --warmup 2 --no-cpu-baseline > $O/bench_c4_b.json 2> $O/bench_c4_b.err
tail -1 $O/bench_c4_b.json
bash profiles/collect_r3_c4.sh $O/prof_c4
python3 profiles/summarize.py $O/prof_c4 --expand k_rexpand --steps 6 --out $O/r3_c4_profile_summary.json
