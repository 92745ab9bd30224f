# GAE hand-off timeline (trace build) and a stagger sweep of the production kernel
DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so timeout -k 10 120 python tools/gae_trace.py > gpurun_out/gt.txt 2>&1 || exit 1
for s in 640 0 320 960 640; do
  echo "stagger $s" >> gpurun_out/gb.txt
  DPPO_GAE_STAGGER=$s timeout -k 10 60 python tools/gae_bench.py >> gpurun_out/gb.txt 2>&1 || exit 1
done
