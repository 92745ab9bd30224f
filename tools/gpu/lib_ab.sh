#!/bin/bash
# A/B of libdppo builds on the default bench workload:
#   bash tools/gpu/lib_ab.sh "<lib names under diamond-ppo_amd/build, 'main' = the shipped one>" [reps] [config]
# then one LDS-counter pass per build (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE of the minibatch kernel).
set -o pipefail
LIBS=$1; REPS=${2:-2}; CFG=${3:-cartpole4096}
R=$(pwd)
mkdir -p gpurun_out/lib_ab
libpath() { [ "$1" = main ] && echo "$R/diamond-ppo_amd/diamond/libdppo.so" || echo "$R/diamond-ppo_amd/build/libdppo_$1.so"; }
for r in $(seq $REPS); do
  for L in $LIBS; do
    DPPO_LIB=$(libpath $L) timeout -k 10 200 python bench.py --config $CFG --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > gpurun_out/lib_ab/$L.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/lib_ab/$L.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$L', d['value'], d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'eval', k['eval']['us_avg'], 'radam', k.get('reduce_adam',{}).get('us_avg'))"
  done
done
cd /tmp && export TMPDIR=/tmp
for L in $LIBS; do
  D=$R/gpurun_out/lib_ab/pmc_$L
  DPPO_LIB=$(libpath $L) timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
    --output-format csv -d $D -o p -- python3 $R/bench.py --config $CFG --no-extra --no-cpu-baseline --no-gae-roofline --steps 2 --warmup 1 > $D.log 2>&1 || exit 1
  python3 - "$D" "$L" <<'PY'
import csv, glob, re, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for row in csv.DictReader(open(f)):
    k = row["Kernel_Name"]
    if "mbw_kernel" not in k and "mb_kernel" not in k and "eval_kernel" not in k: continue
    m = re.search(r"(\w+_kernel(<[^(]*>)?)", k)
    k = m.group(1) if m else k[:60]
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    n[(k, row["Counter_Name"])] += 1
for k, c in acc.items():
    d = {m: v / n[(k, m)] for m, v in c.items()}
    print(sys.argv[2], k, "conflict/active %.1f%%" % (100 * d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1)),
          "VALU/MFMA %.2f" % (d["SQ_INSTS_VALU"] / max(d["SQ_INSTS_MFMA"], 1)), "LDS insts %.0f" % d["SQ_INSTS_LDS"], "wait_lds %.0f" % d["SQ_WAIT_INST_LDS"])
PY
done
