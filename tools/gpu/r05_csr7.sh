#!/bin/bash
# Walk records (fill writes one 16-B record per position on the packed layout): the resolution
# in walk mode (packed and public forms), the global lists from swap targets, then the member
# lists at world 2 / 4 / 8 and their kernel split at world 8.
set -o pipefail
O=gpurun_out/csr7; mkdir -p $O
DPPO_PERM_WALK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dataparallel.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fisher_yates or resolution or swap_targets or c5_full_size or global" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/csr_bench.py --walk 1 2>&1 | grep -v amdgpu.ids
bash tools/gpu/r05_lists_prof.sh
timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0, 'tools'); import gmb_cap as g
print('walk records: global lists ms', {w: round(g.global_lists_ms(w), 3) for w in (2, 4, 8)})
" 2>&1 | grep -v amdgpu.ids
