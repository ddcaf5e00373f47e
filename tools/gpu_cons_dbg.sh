#!/bin/bash
# transRNorm wave kernel: kernel time with phases skipped (KB2E_CONS_DBG bits; timing only, wrong results)
set -o pipefail
TAG=${1:-consdbg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for D in ${DBGS:-0 1 2 4 8 15}; do
  KB2E_CONS_DBG=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/t$D -o run --output-format csv -- \
    python3 bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/t$D.log 2>&1 || { echo "trace $D failed"; exit 1; }
  f=$(find /tmp/t$D -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$D" >> $OUT/summary.txt <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if "transr" in x["Name"] or "rpar" in x["Name"]:
        print("dbg", sys.argv[2], x["Name"].split("(")[0][-45:], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1),
              round(float(x["MinNs"]) / 1e3, 1), round(float(x["MaxNs"]) / 1e3, 1))
PY
  rm -rf /tmp/t$D
done
cat $OUT/summary.txt | grep cons
