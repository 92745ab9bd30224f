# Heavy chunks scanned first: standalone / chained draw, gmb_cap, the draw inside the C5 learn.
set -o pipefail
O=gpurun_out/heavy; mkdir -p $O
timeout -k 10 300 python tools/perm_par_bench.py --threads 12,16 --reps 4 --chain 10 --out $O/draw.json > $O/draw.log 2>&1 || { tail -5 $O/draw.log; exit 1; }
tail -1 $O/draw.log
timeout -k 10 400 python tools/gmb_cap.py --out $O/gmb_cap.json > $O/gmb_cap.log 2>&1 || { tail -5 $O/gmb_cap.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/gmb_cap.json'))
for r in d['rows']: print(r['world'], 'serial', r['host_draw_ms_serial'], 'par', r['host_draw_ms_parallel'], 'chained', r['host_draw_ms_parallel_chained'], 'dev', r.get('device_ms_per_learn_global'), 'cap iso', r.get('speedup_cap_parallel_draw'), 'cap chained', r.get('speedup_cap_parallel_chained_draw'))"
for r in 1 2; do
timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 --warmup 2 > $O/c5.$r.json 2> $O/c5.$r.err || exit 1
python3 -c "import json;d=json.loads(open('$O/c5.$r.json').read().strip().splitlines()[-1]);print('C5', round(d['value']/1e6,1), d['ms_per_step'], d['host_ms_per_step'])"
done
