#!/bin/bash
# Round 6: C3 host-path variants on whatever box this lands on (batch 6 / lib A/B boxes were
# host-bound at ~230 M env-steps/s with either library): default; 4 swap workers; no twist
# producer; unpinned pool; swaps on the device (targets-only host draws), 2 interleaved reps.
set -o pipefail
O=gpurun_out/r06host; mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > $O/$tag.json 2>/dev/null || return 1
  python3 -c "import json;d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);h=d['host_ms_per_step'];print('$tag', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'perms', h['perms'], 'draw', h['draw'], 'slot', h['slot_wait'], 'enq', h['enqueue'], d['host_placement'])"
}
nproc; cat /proc/loadavg
for r in 1 2; do
  run base_$r DPPO_X=0 || exit 1
  run w4_$r DPPO_PERM_WORKERS=4 || exit 1
  run noring_$r DPPO_PERM_RING=0 || exit 1
  run nopin_$r DPPO_PERM_PIN=0 || exit 1
  run dev_$r DPPO_PERM_DEVICE=1 || exit 1
  cat /proc/loadavg
done
