# The parallel draw inside the C5 one-GPU learn (its look-ahead drafts draw while the device runs
# and the launching thread waits): helper placement 0 (scheduler) / 1 (cores after the drawing
# thread's) / 2 (cores from the far end of the mask), 2 reps each; then gmb_cap per placement.
set -o pipefail
O=gpurun_out/pin2; mkdir -p $O
for r in 1 2; do for P in 0 1 2; do
  DPPO_PERM_PAR_PIN=$P timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 --warmup 2 > $O/c5_p$P.$r.json 2> $O/c5_p$P.$r.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/c5_p$P.$r.json').read().strip().splitlines()[-1]);print('pin=$P rep$r C5', round(d['value']/1e6,1), d['ms_per_step'], 'host', d['host_ms_per_step'])"
done; done
for P in 0 1 2; do
  DPPO_PERM_PAR_PIN=$P timeout -k 10 300 python tools/gmb_cap.py --no-gpu --out $O/gmb_p$P.json > $O/gmb_p$P.log 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('$O/gmb_p$P.json'));print('pin=$P standalone draw', d['rows'][0]['host_draw_ms_parallel'])"
done
