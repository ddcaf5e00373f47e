#!/bin/bash
# K5 quick check (n > 64 parity tests + bench), the pipelined chain's phase
# counters at K5, then the TransH profile (bench + trace + PMC).
set -o pipefail
bash tools/gpu_k5quick.sh r21_k5q6 || exit 1
OUT=gpurun_out/r21_k5q6
KB2E_RPAR_STATS=1 timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 10 --warmup 3 > $OUT/k5_stats.json 2> $OUT/k5_stats.err || { echo "k5 stats failed $?"; tail -5 $OUT/k5_stats.err; exit 1; }
grep "pipelined" $OUT/k5_stats.err | tail -1
bash tools/gpu_profile.sh r21_transh parallel --config transh_fb15k || exit 1
bash tools/gpu_k5_trace.sh r21_k5trace5 || exit 1
