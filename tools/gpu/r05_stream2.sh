# GAE data-movement ceiling variants (tools/probe/stream_probe2.hip) under rocprofv3 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/stream2; mkdir -p $O
for N in 8192 65536; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt$N -o kt -- python3 tools/probe/stream_probe2.py $N > $O/run$N.log 2>&1 || { tail -5 $O/run$N.log; exit 1; }
f=$(find $O/kt$N -name "*kernel_trace.csv" | head -1)
python3 - "$f" $N <<'PY'
import csv, sys, collections, re
rows = list(csv.DictReader(open(sys.argv[1])))
keys = rows[0].keys()
gcol = next(k for k in keys if k.lower().startswith('grid_size') or k.lower() == 'grid_size_x' or k.lower()=='grid_size')
d = collections.defaultdict(list)
for r in rows:
    m = re.search(r'stream2_kernel<(\d+)>', r['Kernel_Name'])
    if not m: continue
    d[(int(m.group(1)), int(r[gcol]) // 256)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
N = int(sys.argv[2]); B = 22 * 128 * N
for (mode, grid), v in sorted(d.items()):
    v = sorted(v)[len(v) // 8:]  # drop the warm-up tail
    med = v[len(v) // 2]
    print('N=%d mode=%d (nt=%d x2=%d xcd=%d) grid=%d: median %.2f us min %.2f us -> %.0f GB/s' % (N, mode, mode & 1, (mode >> 1) & 1, (mode >> 2) & 1, grid, med, v[0], B / med / 1e3))
PY
done
