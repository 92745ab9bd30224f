#!/bin/bash
# 16-B observation loads gated on host-checked alignment: eval / pack parity incl. 4-B aligned
# buffers, then the C3 / C2 bench lines.
set -o pipefail
O=gpurun_out/q4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_eval_reuse.py tests/test_gpu_parity.py tests/test_gpu_rollout_ckpt.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for C in lunar8192 cartpole4096; do
  timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/$C.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'eval', k['eval']['us_avg'], 'pack', k['pack']['us_avg'], 'grad', k['grad']['us_avg'], d['roofline']['frac'])"
done
