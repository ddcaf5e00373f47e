#!/bin/bash
# transRNorm chain: parity tests (chain + Jacobi forms) and the chain's phase counters on the bench.
set -o pipefail
OUT=gpurun_out/${1:-cq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py -v --timeout 120 --timeout-method thread -k transr > $OUT/par.log 2>&1; tail -1 $OUT/par.log; grep -E "^FAILED" $OUT/par.log | head -10
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 --seed-epochs 5 > $OUT/bench_stats.json 2> $OUT/bench_stats.err && grep "rpar_cons chunk" $OUT/bench_stats.err | tail -2 &&
python -c "import json;d=json.load(open('$OUT/bench_stats.json'));print(d['value'], d['roofline']['kernels_avg_us'])"
