#!/bin/bash
# kernel stats of the PARALLEL TransR bench under two settings of one env var: tools/gpu_trace_ab.sh TAG VAR V1 V2
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for V in "$@"; do
  env $VAR=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/tr_$V -o run --output-format csv -- \
    python3 bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/trace_$V.log 2>&1 || { echo "trace $V failed"; exit 1; }
  f=$(find /tmp/tr_$V -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$VAR=$V" >> $OUT/summary.txt <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if "transr" in x["Name"] or "rpar" in x["Name"]:
        print(sys.argv[2], x["Name"].split("(")[0][-48:], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1))
PY
  rm -rf /tmp/tr_$V
done
cat $OUT/summary.txt
