# full bench.py (main + configs_extra) under host-placement settings
for e in "A=0" "DPPO_PERM_PIN=1" "DPPO_PERM_PIN=0"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-gae-roofline > gpurun_out/fab.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/fab.json').read().strip().splitlines()[-1])
print('$e main', round(d['value']/1e6,1), d['host_ms_per_step']['draw'])
for k,v in d['configs_extra'].items(): print('   ', k, round(v['value']/1e6,1), v['ms_per_step'], v['device_ms_per_step'], v['host_ms_per_step']['draw'])"
done
