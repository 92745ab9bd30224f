#!/bin/bash
# Round 6: is the C3 host slowdown of batch 6 in the library?  The current libdppo.so against the
# batch-4 build (tools/ab_lib/libdppo_527bb01.so, 286 M env-steps/s then), 3 interleaved pairs.
set -o pipefail
O=gpurun_out/r06lib; mkdir -p $O
for r in 1 2 3; do for V in new old; do
  if [ $V = old ]; then export DPPO_LIB=$GRAFT_REPO_ROOT/tools/ab_lib/libdppo_527bb01.so; else unset DPPO_LIB; fi
  timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > $O/c3_${V}_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_${V}_$r.json').read().strip().splitlines()[-1]);h=d['host_ms_per_step'];print('$V rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'perms', h['perms'], 'draw', h['draw'], 'dev', d['device_ms_per_step'], d['host_placement'])"
done; done
