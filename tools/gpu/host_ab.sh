# host-side A/B on one box: permutation pool placement (DPPO_PERM_PIN 2 = an L3 other than the
# main thread's, 1 = the caller's L3, 0 = one thread)
B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --no-kernel-timing --steps 40 --warmup 5"
run() {
  E="$1"; X="$2 $3"
  timeout -k 10 200 env $E $B $X > gpurun_out/hab.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/hab.json').read().strip().splitlines()[-1]); print('$*', round(d['value']/1e6,1), d['ms_per_step'], d['host_ms_per_step'])"
}
for c in cartpole4096 lunar8192; do
  for p in 2 0 2 0; do run DPPO_PERM_PIN=$p --config $c; done
done
