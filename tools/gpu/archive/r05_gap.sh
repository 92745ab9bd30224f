# Chained draws with idle gaps between them (0 / 5 / 19 ms): is the in-learn slowdown the gaps?
set -o pipefail
O=gpurun_out/gap; mkdir -p $O
for g in 0 5 19 0 19; do
  timeout -k 10 300 python tools/perm_par_bench.py --threads 12 --reps 1 --chain 12 --gap-ms $g > $O/g$g.log 2>&1 || { tail -3 $O/g$g.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/g$g.log').read().strip().splitlines()[-1]);print('gap $g ms: chained median', d['chained_ms_median'], 'min', d['chained_ms_min'])"
done
