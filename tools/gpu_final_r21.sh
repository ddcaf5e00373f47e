#!/bin/bash
# Round-4 closing run: the whole GPU suite, the default bench line (K4, with the
# CPU baseline), the K5 line, and a K5 A/B of the tile LDS budget (St = 8).
set -o pipefail
OUT=gpurun_out/${1:-r21_final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/gpu_tests.log | head -20; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed $?"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print('default',d['value'],d['ms_per_step'],d['roofline']['frac'])"
timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_bench.json 2> $OUT/k5_bench.err || { echo "k5 bench failed $?"; tail -5 $OUT/k5_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_bench.json'));print('K5',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
KB2E_RPAR_TILE_KB=96 timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_st8.json 2> $OUT/k5_st8.err || { echo "k5 st8 bench failed $?"; tail -5 $OUT/k5_st8.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_st8.json'));print('K5 St8',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
