#!/bin/bash
# Buckets heap-sorted past 32 steps + the explicit-scratch C-ABI: resolution tests (both scratch
# forms, adversarial targets), the learn-level resolution tests, C5 A/B, the microbench both forms.
set -o pipefail
O=gpurun_out/csr6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dataparallel.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fisher_yates or resolution or swap_targets or c5_full_size or lookahead or cartpole_decay or cheetah_small" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for M in 1 0; do
  DPPO_PERM_CSR=$M timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 > $O/c5.$M.$r.json 2>$O/c5.$M.$r.err || { tail -5 $O/c5.$M.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c5.$M.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('c5 csr=$M rep$r', round(d['value']/1e6,2), d['ms_per_step'], {c: round(v['ms_total']/v['launches'],3) for c, v in k.items() if c in ('perm','grad','eval')})"
done; done
timeout -k 10 200 python3 tools/csr_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python3 tools/csr_bench.py --public 2>&1 | grep -v amdgpu.ids
