# Per-chunk timings of the parallel draw inside the C5 one-GPU learn (DPPO_PAR_DBG_CHUNKS=1).
set -o pipefail
O=gpurun_out/insitu; mkdir -p $O
DPPO_PAR_DBG_CHUNKS=1 timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --no-kernel-timing --steps 8 --warmup 2 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
python3 - <<'PY'
import re, json
lines = [l for l in open('gpurun_out/insitu/c5.err') if l.startswith('chunk')]
rows = []
for l in lines:
    m = re.search(r'words (\d+) us (\d+) jump (\d+) recs (\d+) raw (\d+) scalar (\d+) W (-?\d+) tsc/word: loop ([\d.]+) twist ([\d.]+)', l)
    rows.append([float(x) for x in m.groups()])
# group into draws of 24 chunks
C = 24
for i in range(0, len(rows) - C + 1, C):
    d = rows[i:i + C]
    us = sorted(r[1] for r in d); tw = sorted(r[8] for r in d); lp = sorted(r[7] for r in d)
    print('draw %d: chunk us min %.0f med %.0f max %.0f | twist tsc/w med %.2f max %.2f | loop tsc/w med %.2f max %.2f | jump max %.0f' % (i // C, us[0], us[C // 2], us[-1], tw[C // 2], tw[-1], lp[C // 2], lp[-1], max(r[2] for r in d)))
d = json.loads(open('gpurun_out/insitu/c5.json').read().strip().splitlines()[-1])
print('C5', round(d['value'] / 1e6, 1), d['ms_per_step'], d['host_ms_per_step'])
PY
