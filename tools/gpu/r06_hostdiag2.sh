set -o pipefail
O=gpurun_out/r06hd; mkdir -p $O
timeout -k 10 200 python -u tools/host_timeline.py --config lunar8192 --learns 24 > $O/timeline2.txt 2>&1 || { tail -20 $O/timeline2.txt; exit 1; }
grep -E "learns|gc_|host_seconds" $O/timeline2.txt | head -40
timeout -k 10 200 python -u tools/host_timeline.py --config lunar8192 --learns 24 > $O/timeline3.txt 2>&1 || { tail -20 $O/timeline3.txt; exit 1; }
grep -E "learns|gc_|host_seconds" $O/timeline3.txt | head -40
