#!/bin/bash
# K5 quick check: the TransR n > 64 matrix-core parity tests, then the K5 bench line
set -o pipefail
OUT=gpurun_out/${1:-k5q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 200 --timeout-method thread -k "transr and (100 or 65 or 96 or 112 or 72 or 88 or 128)" > $OUT/par.log 2>&1 || { echo "tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/par.log | head -20; tail -5 $OUT/par.log; exit 1; }
tail -1 $OUT/par.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_k5.py -x -q --timeout 300 --timeout-method thread > $OUT/k5t.log 2>&1 || { echo "k5 tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/k5t.log | head -20; tail -5 $OUT/k5t.log; exit 1; }
tail -1 $OUT/k5t.log
timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_bench.json 2> $OUT/k5_bench.err || { echo "k5 bench failed $?"; tail -5 $OUT/k5_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_bench.json'));print('K5',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
for v in ${K5_AB:-}; do
  env $v timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_ab.json 2> $OUT/k5_ab.err || { echo "k5 A/B bench failed $?"; tail -5 $OUT/k5_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/k5_ab.json'));print('K5 $v',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
done
