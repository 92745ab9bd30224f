# A/B of the host permutation placement: perm micro-bench from a draft thread, then the quick bench
for p in 1 0; do
  echo "pin $p" >> gpurun_out/ab.txt
  DPPO_PERM_PIN=$p python tools/perm_thread_bench.py >> gpurun_out/ab.txt 2>&1
  DPPO_PERM_PIN=$p python tools/perm_thread_bench.py 1048576 >> gpurun_out/ab.txt 2>&1
  for c in cartpole4096 lunar8192; do
    DPPO_PERM_PIN=$p timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --no-kernel-timing --steps 30 --warmup 5 --config $c > gpurun_out/ab_$p_$c.json 2>/dev/null
    python -c "
import json; d=json.loads(open('gpurun_out/ab_$p_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value']/1e6,1), d['ms_per_step'], d['device_ms_per_step'], d['host_ms_per_step'])" >> gpurun_out/ab.txt
  done
done
