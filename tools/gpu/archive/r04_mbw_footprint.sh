#!/bin/bash
# Minibatch-kernel phase traces at two buffer footprints per instantiation: is the C3 dh2 (+gather)
# phase slow because of the 4-action instantiation or because of the 1M-sample record buffer?
set -o pipefail
O=gpurun_out/mbfp; mkdir -p $O
t() {  # config N
  PHASE_CONFIG=$1 PHASE_N=$2 DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=5000 \
    timeout -k 10 200 python tools/mbw_trace.py > $O/$1_$2.txt 2>&1 || { tail $O/$1_$2.txt; exit 1; }
  echo "== $1 N=$2"; grep -v amdgpu.ids $O/$1_$2.txt | grep -E "dh2|dh1|La/Lc|group total|workgroups"
}
t lunar8192 8192 && t lunar8192 2048 && t cartpole4096 4096 && t cartpole4096 16384
