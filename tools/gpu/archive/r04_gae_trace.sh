#!/bin/bash
# GAE hand-off timelines (trace build, loads-landed stamps behind a wait on the chunk's data):
# the exact kernel and the tolerance-mode kernel at N = 8192.
set -o pipefail
mkdir -p gpurun_out/gtr
DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so timeout -k 10 120 python tools/gae_trace.py > gpurun_out/gtr/exact.txt 2>&1 || exit 1
DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so timeout -k 10 120 python tools/gae_trace.py --affine > gpurun_out/gtr/affine.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/gtr/exact.txt; grep -v amdgpu.ids gpurun_out/gtr/affine.txt
