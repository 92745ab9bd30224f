#!/bin/bash
# Round 6: permutation look-ahead depth 3 (4 pinned slots, the new default) against depth 2 (the
# round-5 pipeline) on whatever box this lands on: C3 and C2 learns, 3 interleaved pairs, and the
# look-ahead hit / miss tests under depth 3.
set -o pipefail
O=gpurun_out/r06depth; mkdir -p $O
nproc; cat /proc/loadavg
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do for V in 3 2; do for C in lunar8192 cartpole4096; do
  DPPO_PERM_DEPTH=$V timeout -k 10 300 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > $O/${C}_${V}_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/${C}_${V}_$r.json').read().strip().splitlines()[-1]);h=d['host_ms_per_step'];print('$C depth=$V rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'perms', h['perms'], 'draw', h['draw'], 'slot', h['slot_wait'])"
done; done; done
cat /proc/loadavg
