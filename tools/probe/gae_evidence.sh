# GAE evidence for profiles/ (run on the GPU box via gpurun): the stream probe (same 22 B/element,
# no recurrence; plain and write-through stores) and the GAE kernel at N = 8192 over 16 rotating
# buffer sets (plain and write-through stores), all under rocprofv3 kernel tracing.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/gae${GAE_TAG:-}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/probe -o probe -- python3 $R/tools/probe/stream_probe.py 8192 > $OUT/probe.log 2>&1
echo probe done
for wt in 0 1; do
  DPPO_GAE_WT=$wt timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gae_wt$wt -o gae -- python3 $R/tools/gae_bench.py --N 8192 --reps 4 > $OUT/gae_wt$wt.log 2>&1
  echo gae wt=$wt done
done
