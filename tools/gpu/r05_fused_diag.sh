# The 1-rank fused peer test variants in one pytest process, exchange buffer addresses printed;
# then [coarse] alone.
set -o pipefail
O=gpurun_out/fdiag; mkdir -p $O
export DPPO_PEER_DEBUG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -m gpu -k "one_rank_fused" -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/all4.log 2>&1; echo "all4 rc=$?"
grep -E "dppo peer:|PASSED|FAILED" $O/all4.log
timeout -k 10 300 python -u -m pytest "tests/test_gpu_peer.py::test_peer_exchange_one_rank_fused_step_reproduces_reference_traces[coarse]" -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/coarse.log 2>&1; echo "coarse rc=$?"
grep -E "dppo peer:|PASSED|FAILED" $O/coarse.log
