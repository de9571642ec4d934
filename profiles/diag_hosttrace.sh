mkdir -p gpurun_out/r2at
for v in old slots; do
  SPLENDOR_BEAM_LIB=$PWD/splendor-rl-gym_amd/splendor_amd/variants/lib_$v.so SB_HOST_TRACE=1 timeout -k 10 120 python3 -u profiles/diag_steps.py 16 > gpurun_out/r2at/diag_$v.txt 2>&1
done
