#!/bin/bash
# Partitioned-bucket Fisher-Yates resolution (shuffle.hip csr_*): bit-exact tests of the device
# resolution and the global-minibatch member lists, then C5 on one GPU against the linked-list
# passes (DPPO_PERM_CSR=0), 2 interleaved reps, bench events per kernel class.
set -o pipefail
O=gpurun_out/csr; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dataparallel.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fisher_yates or swap_targets or c5_full_size or lookahead or cartpole_decay or cheetah_small" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for M in 1 0; do
  DPPO_PERM_CSR=$M timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 > $O/c5.$M.$r.json 2>$O/c5.$M.$r.err || { tail -5 $O/c5.$M.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c5.$M.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('c5 csr=$M rep$r', round(d['value']/1e6,2), d['ms_per_step'], {c: (v['ms_total'], v['launches']) for c, v in k.items() if c in ('perm','grad','eval')})"
done; done
