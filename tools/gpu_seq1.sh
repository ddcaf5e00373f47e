#!/bin/bash
# PARALLEL TransR transRNorm chunk kernel: parity tests, bench with its counters,
# and the PARALLEL side of the FB15k-shaped compat seed envelope.
set -o pipefail
OUT=gpurun_out/${1:-seq1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py -x -v --timeout 120 --timeout-method thread > $OUT/par.log 2>&1; rc=$?; tail -5 $OUT/par.log; [ $rc -eq 0 ] || exit $rc
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/bench_stats.json 2> $OUT/bench_stats.err && grep rpar_cons $OUT/bench_stats.err | tail -2 &&
timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/bench.json 2> $OUT/bench.err && head -c 1200 $OUT/bench.json && echo &&
timeout -k 10 400 python -u tools/seed_envelope.py --model R --compat 1 --seeds 7,8,9,10,11 --schedules parallel --out $OUT/R_compat_par.jsonl 2> $OUT/env.err && grep seed $OUT/env.err
