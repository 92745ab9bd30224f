timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mbw.log 2>&1; tail -2 gpurun_out/t_mbw.log
timeout -k 10 200 python bench.py --no-extra --steps 20 --warmup 5 > gpurun_out/b_new.json 2> gpurun_out/b_new.err
DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=20000 timeout -k 10 120 python tools/mbw_trace.py > gpurun_out/mbwt.txt 2>&1; tail -15 gpurun_out/mbwt.txt
python -c "
import json; d=json.loads(open('gpurun_out/b_new.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['ms_per_step'], d['roofline']['us_per_launch'], d['roofline']['frac'], d['kernels']['reduce_adam']['us_avg'])"
