#!/bin/bash
# Per-phase s_memtime trace of the minibatch kernel (timing-only build without VGPR-form MFMA:
# ROCm 7.2's compiler crashes on the trace build with it) on the C2 / C3 / C4 shapes.
set -o pipefail
mkdir -p gpurun_out/trace
for C in ${1:-cartpole4096 lunar8192 cheetah4096}; do
  PHASE_CONFIG=$C DPPO_LIB=${TRACE_LIB:-diamond-ppo_amd/ab/libdppo_trace.so} WARM_LAUNCHES=20000 timeout -k 10 200 python tools/mbw_trace.py > gpurun_out/trace/$C.txt 2>&1 || exit 1
  echo "== $C"; cat gpurun_out/trace/$C.txt | grep -v amdgpu.ids
done
