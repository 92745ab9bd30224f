# Parallel draw: helpers pinned one per physical core (DPPO_PERM_PAR_PIN=1) against the
# scheduler's placement, chained and isolated, 12 / 16 threads; twist rate per chunk.
set -o pipefail
O=gpurun_out/dpin; mkdir -p $O
python3 tools/probe/host_load.py
for P in 0 1 0 1; do
  DPPO_PERM_PAR_PIN=$P DPPO_PAR_DBG_CHUNKS=1 timeout -k 10 300 python tools/perm_par_bench.py --threads 12,16 --reps 3 --chain 10 --out $O/draw_pin$P.json > $O/draw_pin$P.log 2>&1 || { tail -5 $O/draw_pin$P.log; exit 1; }
  python3 -c "
import json,re
s=json.loads(open('$O/draw_pin$P.log').read().strip().splitlines()[-1])
tw=sorted(float(m.group(1)) for m in re.finditer(r'twist ([\d.]+)', open('$O/draw_pin$P.log').read()))
print('pin=$P', 'iso', s['parallel_ms_median'], 'chained', s['chained_ms_median'], 'chained_min', s['chained_ms_min'], 'twist tsc/w median %.2f p90 %.2f max %.2f' % (tw[len(tw)//2], tw[int(len(tw)*0.9)], tw[-1]))"
done
