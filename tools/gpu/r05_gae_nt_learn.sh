# The GAE's non-temporal default (DPPO_GAE_NT=3) against the previous plain accesses (0) in whole
# learns: C3 and C5-on-one-GPU, 2 pairs, bench events (gae, pack, learn).
set -o pipefail
O=gpurun_out/gaentl; mkdir -p $O
for r in 1 2; do for V in 0 3; do for C in lunar8192 c5; do
  DPPO_GAE_NT=$V timeout -k 10 300 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 10 --warmup 2 > $O/$C.$V.$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/$C.$V.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C NT=$V rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'gae', k['gae']['us_avg'], 'pack', k['pack']['us_avg'], 'grad', k['grad']['us_avg'])"
done; done; done
