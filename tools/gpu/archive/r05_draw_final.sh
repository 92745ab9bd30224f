# Parallel draw with pinned helpers (the default): chained / isolated draw times, the
# global-minibatch cap, the C5 one-GPU learn (its draws run on the same pool).
set -o pipefail
O=gpurun_out/dfinal; mkdir -p $O
python3 tools/probe/host_load.py
timeout -k 10 300 python tools/perm_par_bench.py --threads 8,12,16 --reps 3 --chain 12 --out $O/draw.json > $O/draw.log 2>&1 || { tail -5 $O/draw.log; exit 1; }
tail -1 $O/draw.log
timeout -k 10 400 python tools/gmb_cap.py --out $O/gmb_cap.json > $O/gmb_cap.log 2>&1 || { tail -5 $O/gmb_cap.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/gmb_cap.json'))
for r in d['rows']: print(r['world'], 'draw par', r['host_draw_ms_parallel'], 'thr', r['draw_threads'], 'dev', r.get('device_ms_per_learn_global'), 'cap', r.get('speedup_cap_parallel_draw'))"
timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 --warmup 2 > $O/c5.json 2> $O/c5.err || exit 1
python3 -c "import json;d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print('C5', round(d['value']/1e6,1), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'host', d['host_ms_per_step'])"
