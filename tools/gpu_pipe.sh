#!/bin/bash
# PARALLEL TransR / TransH parity tests, then bench A/B of the transRNorm chain
# kernels (pipelined default vs KB2E_RPAR_CHAIN=serial) and of the TransH
# normOrth passes (per relation + serial default vs KB2E_HPAR_ORTH=serial).
set -o pipefail
OUT=gpurun_out/${1:-pipe}
mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 45; do date >> $OUT/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_hits_parity.py -x -v --timeout 120 --timeout-method thread -k "transr or transh or hits" > $OUT/par.log 2>&1 || { echo "parity tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/par.log | head -20; tail -5 $OUT/par.log; exit 1; }
tail -1 $OUT/par.log
for V in pipe; do
  KB2E_RPAR_CHAIN=$V timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/bench_$V.json 2> $OUT/bench_$V.err || { echo "bench $V failed $?"; exit 1; }
done
for V in rel serial; do
  KB2E_HPAR_ORTH=$V timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --config transh_fb15k --steps 100 --warmup 100 > $OUT/benchH_$V.json 2> $OUT/benchH_$V.err || { echo "benchH $V failed $?"; exit 1; }
done
python - "$OUT" <<'PY'
import json, sys
for f in ("bench_pipe", "benchH_rel", "benchH_serial"):
    d = json.load(open(sys.argv[1] + "/" + f + ".json"))
    p = d["schedules"]["parallel"]
    print(f, round(d["value"]), d["roofline"]["kernels_avg_us"], p.get("epoch"), p.get("late_epoch"))
PY
