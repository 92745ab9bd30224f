# Round 5, batch 2: the parallel draw (threads x chunks per thread, EPYC 9575F), the global-
# minibatch scaling cap with the per-rank member-list kernels, exchange latency by buffer memory
# type (2 / 4 processes on the box's GPU), and bench.py --gpus 2 / 8 rehearsed on one GPU.
set -o pipefail
O=gpurun_out/r05b2; mkdir -p $O
for cpt in 1 2; do
  timeout -k 10 300 python tools/perm_par_bench.py --reps 6 --threads 8,12,16 --chunks-per-thread $cpt --out $O/draw_cpt$cpt.json > $O/draw_cpt$cpt.log 2>&1 || { echo "draw cpt=$cpt failed"; tail -5 $O/draw_cpt$cpt.log; exit 1; }
  echo "cpt=$cpt $(tail -1 $O/draw_cpt$cpt.log)"
done
timeout -k 10 400 python tools/gmb_cap.py --out $O/gmb_cap.json > $O/gmb_cap.log 2>&1; echo gmb rc $?; tail -1 $O/gmb_cap.log | cut -c1-3000
for r in 1 2; do for mem in coarse fine uncached; do for w in 2 4; do
  DPPO_PEER_MEM=$mem timeout -k 10 200 python tools/peer_latency.py $w >> $O/latency.txt 2>&1 || { echo "latency $mem $w failed"; tail -5 $O/latency.txt; exit 1; }
  echo "mem=$mem $(tail -1 $O/latency.txt)"
done; done; done
for g in 2 8; do
  DPPO_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus $g --steps 3 --warmup 1 > $O/rehearse$g.json 2> $O/rehearse$g.err || { echo "rehearse $g failed"; tail -20 $O/rehearse$g.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/rehearse$g.json').read().strip().splitlines()[-1]);print($g, json.dumps(d['multi_gpu']))"
done
