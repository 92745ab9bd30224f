# Node-shared draw: the peer / data-parallel GPU tests (incl. the shared-draw equality test), then
# a rehearsed bench.py --gpus 2 (its configs[4] global leg shares the draw between the ranks).
set -o pipefail
O=gpurun_out/share; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_dataparallel.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -40 | cut -c1-150; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
DPPO_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 4 --warmup 1 > $O/rehearse2.json 2> $O/rehearse2.err || { tail -20 $O/rehearse2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/rehearse2.json').read().strip().splitlines()[-1]); mg=d['multi_gpu']
for m in ('local','global'): r=mg['c5_strong_'+m]; print(m, r['update_steps_per_s'], r['ms_per_step'], r['host_ms_per_step'])
print(mg['exchange'])"
