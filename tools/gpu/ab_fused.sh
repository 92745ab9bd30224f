#!/bin/bash
# A/B of the fused minibatch tail (DPPO_FUSED_ADAM set: slab reduction + clip + Adam inside the
# minibatch kernel, one launch per minibatch) against the default two launches, default bench.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in off on; do
    if [ $v = on ]; then export DPPO_FUSED_ADAM=1; else unset DPPO_FUSED_ADAM; fi
    timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > gpurun_out/abf_$v.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/abf_$v.json').read().strip().splitlines()[-1]);k=d['kernels'];print('fused=$v', d['value'], d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'radam', k.get('reduce_adam',{}).get('us_avg'))"
  done
done
