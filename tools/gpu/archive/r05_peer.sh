# Peer exchange: GPU tests (memory types, the fused exchange across the 2^32 wrap, the bench's
# multi_gpu keys), latency A/B of the exchange-buffer memory types, rehearsed --gpus 2 / 8 lines.
set -o pipefail
O=gpurun_out/r05peer; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_peer.py -m gpu -v -x --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2; do for mem in coarse fine uncached; do for w in 2 4; do
  DPPO_PEER_MEM=$mem timeout -k 10 200 python tools/peer_latency.py $w >> $O/latency.txt 2>&1 || { echo "latency $mem $w failed"; tail -5 $O/latency.txt; exit 1; }
  echo "mem=$mem $(tail -1 $O/latency.txt)"
done; done; done
for g in 2 8; do
  DPPO_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus $g --steps 3 --warmup 1 > $O/rehearse$g.json 2> $O/rehearse$g.err || { echo "rehearse $g failed"; tail -20 $O/rehearse$g.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/rehearse$g.json').read().strip().splitlines()[-1]);print($g, json.dumps(d['multi_gpu']))"
done
