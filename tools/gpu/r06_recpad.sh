#!/bin/bash
# Round 6: 64-B discrete records (DPPO_REC_PAD=1) against 48-B ones: parity under the padded layout
# (production + learn traces), then C2 / C3 learns, 3 interleaved pairs, bench events.
set -o pipefail
O=gpurun_out/r06pad; mkdir -p $O
DPPO_REC_PAD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "REC_PAD=1 parity: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for V in 0 1; do for C in lunar8192 cartpole4096; do
  DPPO_REC_PAD=$V timeout -k 10 300 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 3 > $O/$C.$V.$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/$C.$V.$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C PAD=$V rep$rep', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'pack', k['pack']['us_avg'], 'radam', k.get('reduce_adam',{}).get('us_avg'))"
done; done; done
