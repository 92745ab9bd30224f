# The parallel draw back to back (chained, the learner's host-bound regime) at 8 / 12 / 16
# threads, then the global-minibatch cap with the 12-thread default.
set -o pipefail
O=gpurun_out/dchain; mkdir -p $O
python3 tools/probe/host_load.py
timeout -k 10 300 python tools/perm_par_bench.py --threads 8,12,16 --reps 2 --chain 12 --out $O/draw.json > $O/draw.log 2>&1 || { tail -5 $O/draw.log; exit 1; }
tail -1 $O/draw.log
timeout -k 10 400 python tools/gmb_cap.py --out $O/gmb_cap.json > $O/gmb_cap.log 2>&1 || { tail -5 $O/gmb_cap.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/gmb_cap.json'))
for r in d['rows']: print(r['world'], 'draw par', r['host_draw_ms_parallel'], 'thr', r['draw_threads'], 'dev', r.get('device_ms_per_learn_global'), 'cap', r.get('speedup_cap_parallel_draw'))"
python3 tools/probe/host_load.py
