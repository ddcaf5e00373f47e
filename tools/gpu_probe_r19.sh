#!/bin/bash
# r19 probe: the CLI compat-eval test alone (durations), then the transRNorm chain counters on the bench.
set -o pipefail
OUT=gpurun_out/r19b
mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 45; do date >> $OUT/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 280 python -u -m pytest tests/test_gpu_cli.py -x -v --timeout 250 --timeout-method thread --durations=0 -k "eval" > $OUT/cli.log 2>&1 || { echo "cli test failed $?"; tail -30 $OUT/cli.log; exit 1; }
tail -8 $OUT/cli.log
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 --seed-epochs 5 > $OUT/bench_stats.json 2> $OUT/bench_stats.err || { echo "bench stats failed $?"; tail $OUT/bench_stats.err; exit 1; }
grep "rpar_cons chunk" $OUT/bench_stats.err | tail -2
cat $OUT/bench_stats.json
