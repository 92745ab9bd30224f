# Parallel draw (pinned helpers, 12 threads default), serial reference on resident pages; the
# global-minibatch cap with isolated and chained draws.
set -o pipefail
O=gpurun_out/dfinal2; mkdir -p $O
python3 tools/probe/host_load.py
timeout -k 10 300 python tools/perm_par_bench.py --threads 8,12,16 --reps 4 --chain 10 --out $O/draw.json > $O/draw.log 2>&1 || { tail -5 $O/draw.log; exit 1; }
tail -1 $O/draw.log
timeout -k 10 400 python tools/gmb_cap.py --out $O/gmb_cap.json > $O/gmb_cap.log 2>&1 || { tail -5 $O/gmb_cap.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/gmb_cap.json'))
for r in d['rows']: print(r['world'], 'serial', r['host_draw_ms_serial'], 'par', r['host_draw_ms_parallel'], 'chained', r['host_draw_ms_parallel_chained'], 'dev', r.get('device_ms_per_learn_global'), 'cap iso', r.get('speedup_cap_parallel_draw'), 'cap chained', r.get('speedup_cap_parallel_chained_draw'))"
