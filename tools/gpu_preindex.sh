#!/bin/bash
# The -m gpu suite, then the default bench with and without the prebuilt next-epoch index.
set -o pipefail
TAG=${1:-pre}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for S in 20 100; do
  KB2E_NO_PREINDEX=1 timeout -k 10 300 python bench.py --steps $S --warmup 5 > $OUT/bench_off_$S.json 2> $OUT/bench_off_$S.err || { echo "bench off failed"; tail $OUT/bench_off_$S.err; exit 1; }
  timeout -k 10 300 python bench.py --steps $S --warmup 5 > $OUT/bench_on_$S.json 2> $OUT/bench_on_$S.err || { echo "bench on failed"; tail $OUT/bench_on_$S.err; exit 1; }
  echo "steps $S off: $(python3 -c "import json;d=json.load(open('$OUT/bench_off_$S.json'));print(d['value'],d['ms_per_step'])")  on: $(python3 -c "import json;d=json.load(open('$OUT/bench_on_$S.json'));print(d['value'],d['ms_per_step'])")"
done
for C in transe_fb15k transh_fb15k; do
  timeout -k 10 300 python bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo "bench $C failed"; tail $OUT/bench_$C.err; exit 1; }
  echo "$C $(python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pre_tr -o run --output-format csv -- \
  python3 bench.py --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find /tmp/pre_tr -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(x["Name"].split("(")[0][-48:], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), round(float(x["TotalDurationNs"]) / 1e6, 2))
PY
