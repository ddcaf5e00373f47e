#!/bin/bash
# Kernel timeline of the driver-style bench (K=20 from an epoch boundary): gpurun_out/<tag>/timeline.txt
set -o pipefail
TAG=${1:-tl}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl -o run --output-format csv -- \
  python3 bench.py --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "trace failed"; tail $OUT/bench.log; exit 1; }
f=$(find /tmp/tl -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/timeline.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
print(list(rows[0].keys()))
idx = [i for i, r in enumerate(rows) if "cons_wave" in r["Kernel_Name"]]
a = idx[-21] if len(idx) > 21 else idx[0]
# back up to include the boundary work before the first timed batch
t0 = int(rows[a]["Start_Timestamp"]) - 400000
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0:
        continue
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kb2e::", "")[:56]
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} q{r.get('Queue_Id', '?'):>3} s{r.get('Stream_Id', '?'):>3} {n}")
PY
tail -5 $OUT/timeline.txt
