# A/B of the MT19937 producer ring (DPPO_PERM_RING) in bench.py, C2 and C3
B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --no-kernel-timing --steps 30 --warmup 5"
for c in cartpole4096 lunar8192; do
  for r in 1 0 1 0; do
    DPPO_PERM_RING=$r timeout -k 10 200 $B --config $c > gpurun_out/rab.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/rab.json').read().strip().splitlines()[-1]); print('$c ring=$r', round(d['value']/1e6,1), d['ms_per_step'], d['host_ms_per_step']['draw'], d['host_ms_per_step']['slot_wait'])"
  done
done
