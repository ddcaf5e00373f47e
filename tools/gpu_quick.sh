#!/bin/bash
# Quick GPU check: the evaluator and PARALLEL TransR / TransH parity tests, one bench line.
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 45; do date >> $OUT/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_parallel.py -x -v --timeout 120 --timeout-method thread -k "eval or transr or transh" > $OUT/par.log 2>&1 || { echo "tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/par.log | head -20; tail -5 $OUT/par.log; exit 1; }
tail -1 $OUT/par.log
timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; exit 1; }
python - "$OUT" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench.json"))
p = d["schedules"]["parallel"]
print(round(d["value"]), d["roofline"]["kernels_avg_us"], p.get("epoch"), p.get("late_epoch"))
PY
