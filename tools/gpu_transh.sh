#!/bin/bash
# PARALLEL TransH on the GPU box: tests, bench, kernel stats.  Logs: gpurun_out/<tag>/
set -o pipefail
TAG=${1:-transh}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_transh.py -x -v --timeout 120 --timeout-method thread -k transh \
    > $OUT/pytest.log 2>&1 || { echo "pytest failed $?"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 bench.py --config transh_fb15k --only --no-cpu-baseline --steps 300 --warmup 100 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/trh -o run --output-format csv -- \
    python3 bench.py --config transh_fb15k --only --no-cpu-baseline --no-epoch --steps 300 --warmup 100 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
find /tmp/trh -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 - "$OUT" <<'PY'
import csv, json, sys
d = sys.argv[1]
b = json.load(open(d + "/bench.json"))
print("value", round(b["value"]), "ms/step", round(b["ms_per_step"], 4), "frac", round(b["roofline"]["frac"], 4),
      "epoch", b["schedules"]["parallel"]["epoch"])
for x in list(csv.DictReader(open(d + "/kernel_stats.csv")))[:12]:
    print(" ", x["Name"].split("(")[0][-50:], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1))
PY
