#!/bin/bash
# Round 6 A/B: the minibatch (mbwave) and eval (mlp) kernels under other LLVM scheduler settings;
# each variant library goes to diamond-ppo_amd/ab_r06/libdppo_<tag>.so (hazard-audited like the default)
set -e
cd "$(dirname "$0")/../diamond-ppo_amd"
H=/opt/rocm/bin/hipcc
BASE="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -I../include -Icsrc -Wall -Wno-unused-function -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form"
build() {  # tag, extra flags
  tag=$1; shift
  mkdir -p ab_r06; d=ab/sched/$tag; mkdir -p $d
  $H $BASE "$@" -c csrc/mbwave.hip -o $d/mbwave.o
  $H $BASE "$@" -c csrc/mlp.hip -o $d/mlp.o
  $H $BASE "$@" --cuda-device-only -S csrc/mbwave.hip -o $d/mbwave.s
  python3 ../tools/mfma_hazards.py $d/mbwave.s > $d/hazards.txt || { echo "$tag: hazard audit failed"; cat $d/hazards.txt | tail -5; return 1; }
  objs=""
  for o in gae mbstep optim capi perm permpar shuffle gru peer; do objs="$objs build/$o.o"; done
  $H -shared -fPIC --offload-arch=gfx950 -o ab_r06/libdppo_$tag.so $d/mbwave.o $d/mlp.o $objs -L/opt/rocm/lib -lrccl -pthread -Wl,-rpath,/opt/rocm/lib
  echo "$tag ok"
}
build maxilp -mllvm -amdgpu-sched-strategy=max-ilp &
build bias0 -mllvm -amdgpu-schedule-metric-bias=0 &
wait
