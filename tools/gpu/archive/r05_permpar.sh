set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/perm_par_bench.py --reps 5 --threads 4,8,12,16 --out gpurun_out/perm_par_r05a.json > gpurun_out/perm_par_r05a.log 2>&1 && tail -1 gpurun_out/perm_par_r05a.log && \
DPPO_PERM_PAR_MIN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "learn_matches_reference_trace or lookahead" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_pytest.log 2>&1; echo pytest rc $?; tail -2 gpurun_out/r05a_pytest.log; \
timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 6 --warmup 2 > gpurun_out/c5_par.json 2> gpurun_out/c5_par.err; echo bench rc $?; python -c "
import json;d=json.loads(open('gpurun_out/c5_par.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['device_ms_per_step'],d['host_ms_per_step'],d['kernels'].get('perm'))"
