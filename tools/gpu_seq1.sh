#!/bin/bash
# PARALLEL TransR transRNorm chain: parity tests, bench with its counters (KB2E_RPAR_STATS),
# bench, and the PARALLEL side of the FB15k-shaped compat seed envelope.
set -o pipefail
OUT=gpurun_out/${1:-seq1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py -v --timeout 120 --timeout-method thread > $OUT/par.log 2>&1; tail -3 $OUT/par.log; grep -E "^FAILED|Error:" $OUT/par.log | head -10
KB2E_RPAR_CONS=jacobi timeout -k 10 120 python -u -m pytest tests/test_gpu_parallel.py -v --timeout 120 --timeout-method thread -k "chain_widths" > $OUT/par17j.log 2>&1; tail -1 $OUT/par17j.log
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 --seed-epochs 5 > $OUT/bench_stats.json 2> $OUT/bench_stats.err && grep "rpar_cons chunk" $OUT/bench_stats.err | tail -1 &&
timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/bench.json 2> $OUT/bench.err && python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['roofline']['frac'], d['roofline']['kernels_avg_us'], d['schedules'])" &&
timeout -k 10 400 python -u tools/seed_envelope.py --model R --compat 1 --seeds 7,8,9,10,11 --schedules parallel --out $OUT/R_compat_par.jsonl 2> $OUT/env.err && grep seed $OUT/env.err
