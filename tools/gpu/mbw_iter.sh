# one iteration of minibatch-kernel work: parity, trace of the phases, quick bench
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mbw.log 2>&1 || { tail -30 gpurun_out/t_mbw.log; exit 1; }
tail -2 gpurun_out/t_mbw.log
DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=20000 timeout -k 10 120 python tools/mbw_trace.py > gpurun_out/mbwt.txt 2>&1 || exit 1
tail -6 gpurun_out/mbwt.txt
timeout -k 10 200 python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 30 --warmup 5 > gpurun_out/q_c2.json 2> gpurun_out/q_c2.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/q_c2.json').read().strip().splitlines()[-1]); print('c2', round(d['value']/1e6,1), d['ms_per_step'], d['device_ms_per_step'], d['host_work_ms_per_step'], d['roofline']['us_per_launch'], d['roofline']['frac'], d['kernels']['reduce_adam']['us_avg'])"
