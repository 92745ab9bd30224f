#!/bin/bash
# GAE tile-width / mode timings and timelines, and the global-minibatch draw cap (round 3).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 env DPPO_GAE_E=64 python tools/gae_sizes.py > gpurun_out/r03_gae_e64.jsonl 2>&1 || exit 1
grep N gpurun_out/r03_gae_e64.jsonl
export DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so
timeout -k 10 100 python tools/gae_trace.py > gpurun_out/r03_gae_trace_exact.txt 2>&1 || exit 1
timeout -k 10 100 python tools/gae_trace.py --affine > gpurun_out/r03_gae_trace_affine.txt 2>&1 || exit 1
unset DPPO_LIB
grep -v amdgpu.ids gpurun_out/r03_gae_trace_exact.txt gpurun_out/r03_gae_trace_affine.txt
for ring in 0 1; do
  DPPO_PERM_RING=$ring timeout -k 10 300 python tools/gmb_cap.py > gpurun_out/r03_gmb_cap_ring$ring.json 2> gpurun_out/r03_gmb_cap_ring$ring.err || exit 1
  cat gpurun_out/r03_gmb_cap_ring$ring.json
done
