# reduce_adam with non-temporal slab reads (ab/libdppo_ranT.so) against the default, C3 / C2, 2 pairs.
set -o pipefail
O=gpurun_out/rant; mkdir -p $O
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/ab/libdppo_$1.so; }
for C in lunar8192 cartpole4096; do for r in 1 2; do for L in main ranT; do
  DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'radam', k['reduce_adam']['us_avg'], 'grad', k['grad']['us_avg'])"
done; done; done
