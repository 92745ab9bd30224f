#!/bin/bash
# Production-size soak (bit-identical back-to-back learns, clean error word), then the
# reference-exact scaling cap with the partitioned buckets (tools/gmb_cap.py), and the member
# lists with the linked lists (DPPO_PERM_CSR=0) beside it.
set -o pipefail
O=gpurun_out/csrgmb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_soak.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/soak.log 2>&1
rc=$?; tail -6 $O/soak.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/gmb_cap.py --out $O/gmb_cap_csr.json > $O/gmb.log 2>&1 || { tail -5 $O/gmb.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/gmb_cap_csr.json'))
for r in d['rows']: print({k: r.get(k) for k in ('world','host_draw_ms_parallel','host_draw_ms_parallel_chained','device_ms_share_local','device_ms_global_lists','device_ms_per_learn_global','speedup_cap_parallel_draw','speedup_cap_parallel_chained_draw')})
"
DPPO_PERM_CSR=0 timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0, 'tools'); import gmb_cap as g
print('linked lists: global lists ms', {w: round(g.global_lists_ms(w), 3) for w in (2, 4, 8)})
" 2>&1 | grep -v amdgpu.ids
