#!/bin/bash
# transRNorm kernel on the GPU box: PARALLEL TransR tests, round statistics,
# kernel stats, bench (register-resident kernel vs KB2E_RPAR_CONS=tile).  Logs: gpurun_out/<tag>/
set -o pipefail
TAG=${1:-cons}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py -x -v --timeout 120 --timeout-method thread -k transr \
    > $OUT/pytest.log 2>&1 || { echo "pytest failed $?"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python3 tools/probe_rounds.py compat 100 > $OUT/rounds.log 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 300 python3 bench.py --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/bench_wave.json 2> $OUT/bench_wave.err || { echo "bench failed"; exit 1; }
KB2E_RPAR_FUSE=0 timeout -k 10 300 python3 bench.py --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/bench_nofuse.json 2> $OUT/bench_nofuse.err || { echo "bench nofuse failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
echo done
