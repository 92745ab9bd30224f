#!/bin/bash
# A/B of an environment switch on the default bench workload: bash tools/gpu/ab_env.sh VAR [reps]
set -o pipefail
VAR=$1; REPS=${2:-2}
mkdir -p gpurun_out
for r in $(seq $REPS); do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > gpurun_out/ab_${VAR}_$v.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_${VAR}_$v.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$VAR=$v', d['value'], d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'radam', k.get('reduce_adam',{}).get('us_avg'))"
  done
done
