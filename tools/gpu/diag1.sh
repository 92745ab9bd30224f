set -e
B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 30 --warmup 5"
timeout -k 10 200 $B > gpurun_out/d_def.json 2> gpurun_out/d_def.err
DPPO_PERM_DEVICE=1 timeout -k 10 200 $B > gpurun_out/d_dev.json 2> gpurun_out/d_dev.err
DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=20000 timeout -k 10 120 python tools/mbw_trace.py > gpurun_out/mbwt.txt 2>&1
