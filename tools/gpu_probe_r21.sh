#!/bin/bash
# Round-4 probes: the wide chain's parity subset, the K5 and K4 chain kernels' phase
# counters, the ORDERED TransR n = 100 speed, TransR fixed-energy Hits@10 parity.
set -o pipefail
OUT=gpurun_out/${1:-probe_r21}
mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 45; do date >> $OUT/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py -x -v --timeout 300 --timeout-method thread -k "wide or fixed or compat" > $OUT/par.log 2>&1 || { echo "parallel tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/par.log | head -20; exit 1; }
tail -1 $OUT/par.log
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_stats.json 2> $OUT/k5_stats.err || { echo "k5 stats failed $?"; exit 1; }
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/k4_stats.json 2> $OUT/k4_stats.err || { echo "k4 stats failed $?"; exit 1; }
timeout -k 10 300 python -u tools/seed_envelope.py --model R --dim 100 --epochs 2 --seed-epochs 10 --seeds 7 --test 2000 --out $OUT/n100_speed.jsonl > $OUT/n100_speed.log 2>&1 || { echo "n100 speed failed $?"; exit 1; }
timeout -k 10 700 python -u tools/hits_parity.py --model R --compat 0 --epochs 100 --seed-epochs 500 --test 0 > $OUT/hits_R_fixed.json 2> $OUT/hits_R_fixed.err || { echo "hits failed $?"; exit 1; }
echo done
