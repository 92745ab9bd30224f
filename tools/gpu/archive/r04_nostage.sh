#!/bin/bash
# Upper bound of a prebuilt weight image: the minibatch kernel without its prologue weight loads
# (build/libdppo_nostage.so, timing only) against the shipped library, C2 / C3 / C4.
set -o pipefail
O=gpurun_out/r04ns; mkdir -p $O
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for C in cartpole4096 lunar8192 cheetah4096; do
  for r in 1 2; do
    for L in main nostage; do
      DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.loads(open('$O/$C.$L.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', d['value'], 'grad', k['grad']['us_avg'], 'radam', k['reduce_adam']['us_avg'])"
    done
  done
done
