#!/bin/bash
# GAE tile-width / mode timings and timelines, and the global-minibatch draw cap (round 3).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/gae_sizes.py > gpurun_out/r03_gae_e64.jsonl 2>&1 || exit 1
grep N gpurun_out/r03_gae_e64.jsonl; timeout -k 10 200 python -m pytest -q tests/test_gpu_parity.py -k gae -p no:cacheprovider 2>&1 | tail -2
export DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so
timeout -k 10 100 python tools/gae_trace.py > gpurun_out/r03_gae_trace_exact.txt 2>&1 || exit 1
timeout -k 10 100 python tools/gae_trace.py --affine > gpurun_out/r03_gae_trace_affine.txt 2>&1 || exit 1
unset DPPO_LIB
grep -v amdgpu.ids gpurun_out/r03_gae_trace_exact.txt gpurun_out/r03_gae_trace_affine.txt
for ring in 0; do
  DPPO_PERM_TARGETS_RING=$ring timeout -k 10 300 python tools/gmb_cap.py > gpurun_out/r03_gmb_cap_ring$ring.json 2> gpurun_out/r03_gmb_cap_ring$ring.err || exit 1
  cat gpurun_out/r03_gmb_cap_ring$ring.json
done
# C4 on the sample-split kernel (DPPO_MBW_CONT6=1) against the two-team kernel
for v in 0 1; do
  DPPO_MBW_CONT6=$v timeout -k 10 200 python bench.py --config cheetah4096 --no-extra --no-cpu-baseline --no-gae-roofline --steps 10 > gpurun_out/r03_c4_cont6_$v.json 2> gpurun_out/r03_c4_cont6_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r03_c4_cont6_$v.json').read().strip().splitlines()[-1]);print('cont6=$v', d['value'], d['ms_per_step'], d['roofline']['us_per_launch'], d['roofline']['frac'])"
done
DPPO_MBW_CONT6=1 timeout -k 10 200 python -m pytest -q tests/test_gpu_production.py -k "C4 or cheetah or 17" -p no:cacheprovider 2>&1 | tail -3
