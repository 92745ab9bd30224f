# A/B: first-group staging on / off (DPPO_NO_STAGE), same box
B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 30 --warmup 5"
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export DPPO_NO_STAGE=1; else unset DPPO_NO_STAGE; fi
  timeout -k 10 200 $B > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('no_stage=$v', round(d['value']/1e6,1), d['ms_per_step'], d['device_ms_per_step'], d['roofline']['us_per_launch'], d['kernels']['reduce_adam']['us_avg'])"
done
