#!/bin/bash
# GPU check of the wide transRNorm chain (kernels_transr_chainw.hpp): the PARALLEL
# TransR parity tests against oracle/parallel.py, the full-size K5 property test,
# the evaluator tests, and K5 / K4 bench lines with the chain's phase counters.
# usage: tools/gpu_chainw.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-chainw}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parallel.py -x -v --timeout 300 --timeout-method thread -k "transr or transh" > $OUT/par.log 2>&1 || { echo "parallel tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/par.log | head -20; tail -5 $OUT/par.log; exit 1; }
tail -1 $OUT/par.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_k5.py tests/test_gpu_eval.py -x -v --timeout 400 --timeout-method thread > $OUT/k5.log 2>&1 || { echo "k5/eval tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/k5.log | head -20; tail -5 $OUT/k5.log; exit 1; }
tail -1 $OUT/k5.log
KB2E_RPAR_STATS=1 timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_stats.json 2> $OUT/k5_stats.err || { echo "k5 bench failed $?"; tail -5 $OUT/k5_stats.err; exit 1; }
timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_bench.json 2> $OUT/k5_bench.err || { echo "k5 bench failed $?"; tail -5 $OUT/k5_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_bench.json'));print('K5',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/k4_bench.json 2> $OUT/k4_bench.err || { echo "k4 bench failed $?"; tail -5 $OUT/k4_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k4_bench.json'));print('K4',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
KB2E_RPAR_CHAIN=wide timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/k4_wide.json 2> $OUT/k4_wide.err || { echo "k4 wide bench failed $?"; tail -5 $OUT/k4_wide.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k4_wide.json'));print('K4 wide',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
KB2E_RPAR_TGROUP=1 timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_tg1.json 2> $OUT/k5_tg1.err || { echo "k5 tgroup=1 bench failed $?"; tail -5 $OUT/k5_tg1.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_tg1.json'));print('K5 tgroup=1',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
KB2E_RPAR_CHAIN=lockstep timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_lockstep.json 2> $OUT/k5_lockstep.err || { echo "k5 lockstep bench failed $?"; tail -5 $OUT/k5_lockstep.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_lockstep.json'));print('K5 lockstep',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
