#!/bin/bash
# K5 (TransR n=100, 160,000-sample batches) per-kernel times: rocprofv3 kernel
# trace over a short bench run; the stats CSV lands in gpurun_out/<tag>/trace.
set -o pipefail
OUT=gpurun_out/${1:-k5trace}
mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 45; do date >> "$OUT/heartbeat"; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 10 --warmup 3 > "$OUT/trace.log" 2>&1 || { echo "trace failed $?"; tail -5 "$OUT/trace.log"; exit 1; }
f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-90s %6s %12.1f us avg %10.1f" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
