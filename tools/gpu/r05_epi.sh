# Quarter-ownership epilogue of the minibatch kernel: the full GPU suite, then bench A/B against
# the previous library (ab/libdppo_base.so) on C2 / C3 / C4, 2 pairs each, kernel events.
set -o pipefail
O=gpurun_out/epi; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/ab/libdppo_$1.so; }
for C in cartpole4096 lunar8192 cheetah4096; do
  for r in 1 2; do
    for L in base main; do
      DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.$r.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'frac', d['roofline']['frac'])"
    done
  done
done
