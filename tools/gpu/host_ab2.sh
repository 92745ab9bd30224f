B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --no-kernel-timing --steps 40 --warmup 5"
run() {
  E="$1"; X="$2 $3"
  timeout -k 10 200 env $E $B $X > gpurun_out/hab.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/hab.json').read().strip().splitlines()[-1]); print('$*', round(d['value']/1e6,1), d['ms_per_step'], d['host_ms_per_step'])"
}
for v in 1 0 1 0; do run DPPO_SLOTWAIT_MAIN=$v --config cartpole4096; done
run "DPPO_SLOTWAIT_MAIN=1 DPPO_PERM_DEPTH=1" --config cartpole4096
