# A/B of two builds of libdppo on one box (bench kernel table): $1 = alternative library
B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 30 --warmup 5"
for lib in "" "$1" "" "$1"; do
  DPPO_LIB=$lib timeout -k 10 200 $B > gpurun_out/lab.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/lab.json').read().strip().splitlines()[-1]); k=d['kernels']; print('${lib:-default}', round(d['value']/1e6,1), d['ms_per_step'], k['eval']['us_avg'], k['grad']['us_avg'], k['reduce_adam']['us_avg'])"
done
