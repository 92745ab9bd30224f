# Minibatch-kernel record gathers with the non-temporal cache policy (ab/libdppo_gnt.so) against
# the default: production parity under it, then C2 / C3 / C4 / C5, 2 pairs, bench events.
set -o pipefail
O=gpurun_out/gnt; mkdir -p $O
DPPO_LIB=diamond-ppo_amd/ab/libdppo_gnt.so timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/ab/libdppo_$1.so; }
for r in 1 2; do for C in cartpole4096 lunar8192 cheetah4096 c5; do for L in main gnt; do
  st=20; [ $C = c5 ] && st=8
  DPPO_LIB=$(lib $L) timeout -k 10 300 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps $st > $O/$C.$L.$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'radam', k['reduce_adam']['us_avg'], 'grad', k['grad']['us_avg'], 'frac', d['roofline']['frac'])"
done; done; done
