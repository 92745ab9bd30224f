set -o pipefail
mkdir -p gpurun_out/gstats
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "large_mean" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gstats/new.log 2>&1; echo "new rc=$?"; tail -3 gpurun_out/gstats/new.log
DPPO_LIB=diamond-ppo_amd/build/libdppo_base.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "large_mean" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gstats/base.log 2>&1; echo "base(plain fp32 partials) rc=$?"; grep -E "passed|failed" gpurun_out/gstats/base.log | tail -2; grep -E "^E .*assert" gpurun_out/gstats/base.log | head -4
grep -q "passed" gpurun_out/gstats/new.log && ! grep -q "failed" gpurun_out/gstats/new.log || exit 1
bash tools/gpu/gae_ab.sh
