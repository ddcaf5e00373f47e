#!/bin/bash
# wpipe K5 timing: stats default, stats with projections after the walk, bench default
set -o pipefail
OUT=gpurun_out/${1:-wp}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 200 --timeout-method thread -k "wide_chain_windows or compat_chunk_prefix or (fixed and 100)" > $OUT/par.log 2>&1 || { echo "tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/par.log | head -20; tail -5 $OUT/par.log; exit 1; }
tail -1 $OUT/par.log
KB2E_RPAR_STATS=1 timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 10 --warmup 3 > $OUT/k5_stats.json 2> $OUT/k5_stats.err || { echo "k5 stats failed $?"; tail -5 $OUT/k5_stats.err; exit 1; }
grep "pipelined" $OUT/k5_stats.err
KB2E_CONS_DBG=1 KB2E_RPAR_STATS=1 timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 10 --warmup 3 > $OUT/k5_dbg1.json 2> $OUT/k5_dbg1.err || { echo "k5 dbg1 failed $?"; tail -5 $OUT/k5_dbg1.err; exit 1; }
grep "pipelined" $OUT/k5_dbg1.err
timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_bench.json 2> $OUT/k5_bench.err || { echo "k5 bench failed $?"; tail -5 $OUT/k5_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_bench.json'));print('K5',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 20 > $OUT/k4_stats.json 2> $OUT/k4_stats.err || { echo "k4 stats failed $?"; tail -5 $OUT/k4_stats.err; exit 1; }
grep "rpar_cons" $OUT/k4_stats.err | tail -3
