#!/bin/bash
# Per-kernel averages of the PARALLEL TransR bench, per-epoch kernels included: gpurun_out/<tag>/kernels.txt
set -o pipefail
TAG=${1:-ek}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ek -o run --output-format csv -- \
  python3 bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
f=$(find /tmp/ek -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats.csv
python3 - "$f" > $OUT/kernels.txt <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if "transe_" in x["Name"]:
        continue
    print(x["Name"].split("(")[0].replace("void ", "").replace("kb2e::", "")[-50:], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1))
PY
cat $OUT/kernels.txt
