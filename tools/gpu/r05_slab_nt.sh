# Minibatch-kernel slab stores: write-through (default) / write-through + nt / nt, C2 / C3 / C4,
# 2 rounds, bench events.
set -o pipefail
O=gpurun_out/slabnt; mkdir -p $O
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/ab/libdppo_$1.so; }
for r in 1 2; do for C in cartpole4096 lunar8192 cheetah4096; do for L in main slabntsc slabnt; do
  DPPO_LIB=$(lib $L) timeout -k 10 300 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'radam', k['reduce_adam']['us_avg'], 'grad', k['grad']['us_avg'], 'frac', d['roofline']['frac'])"
done; done; done
