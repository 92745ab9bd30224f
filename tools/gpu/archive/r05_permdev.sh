# Device Fisher-Yates resolution: epoch-at-a-time (DPPO_PERM_EPOCHWISE=1) vs all epochs at once at
# C5 one-GPU (4 x 8.4 M targets), parity of the device-shuffle learn traces with it, then the
# global-minibatch scaling cap with the parallel host draw (tools/gmb_cap.py).
set -o pipefail
O=gpurun_out/r05perm; mkdir -p $O
DPPO_PERM_EPOCHWISE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "learn_matches_reference_trace or lookahead" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head; exit $rc; }
for rep in 1 2; do for ew in 0 1; do
  DPPO_PERM_EPOCHWISE=$ew timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 6 --warmup 2 > $O/c5_ew$ew.$rep.json 2> $O/c5_ew$ew.$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/c5_ew$ew.$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];print('epochwise=$ew rep$rep', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms dev', d['device_ms_per_step'], 'perm', k['perm']['us_avg'], 'us draw', d['host_ms_per_step']['draw'])"
done; done
timeout -k 10 400 python tools/gmb_cap.py --out $O/gmb_cap.json > $O/gmb_cap.log 2>&1; echo gmb rc $?; tail -1 $O/gmb_cap.log | cut -c1-3000
