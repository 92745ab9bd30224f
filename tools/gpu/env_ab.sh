# A/B of an environment switch on one box: $1 = VAR=value, $2 = bench config
B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 --config $2"
for e in "A=0" "$1" "A=0" "$1"; do
  env $e timeout -k 10 200 $B > gpurun_out/eab.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/eab.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$e', round(d['value']/1e6,1), d['ms_per_step'], k['grad']['us_avg'], d['roofline']['frac'])"
done
