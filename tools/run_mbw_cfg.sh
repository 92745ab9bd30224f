# parity tests + per-config minibatch-kernel timing (new kernel vs DPPO_MB_LEGACY=1)
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_rollout_ckpt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mbw.log 2>&1; tail -2 gpurun_out/t_mbw.log
for cfg in cartpole4096 lunar8192 cheetah4096; do
  timeout -k 10 200 python bench.py --no-extra --config $cfg --steps 10 --warmup 3 > gpurun_out/b_$cfg.json 2>/dev/null
  DPPO_MB_LEGACY=1 timeout -k 10 200 python bench.py --no-extra --config $cfg --steps 10 --warmup 3 > gpurun_out/b_${cfg}_old.json 2>/dev/null
  python -c "
import json
for n in ['$cfg', '${cfg}_old']:
    d=json.loads(open('gpurun_out/b_'+n+'.json').read().strip().splitlines()[-1])
    print(n, round(d['value']/1e6,1), d['ms_per_step'], d['roofline']['us_per_launch'], d['roofline']['frac'])"
done
