#!/bin/bash
# Round 6: C3 learns with the host-placement guard (busy domains passed over) against CPU order
# only (DPPO_PERM_BY_LOAD=0), 3 interleaved pairs.
set -o pipefail
O=gpurun_out/r06pl; mkdir -p $O
for r in 1 2 3; do for V in 1 0; do
  DPPO_PERM_BY_LOAD=$V timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > $O/c3_${V}_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_${V}_$r.json').read().strip().splitlines()[-1]);h=d['host_ms_per_step'];print('BY_LOAD=$V rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'perms', h['perms'], 'draw', h['draw'], d['host_placement'])"
done; done
