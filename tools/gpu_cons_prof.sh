#!/bin/bash
# transRNorm kernel: round statistics + rocprofv3 kernel stats of the PARALLEL TransR bench.
set -o pipefail
TAG=${1:-consprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/probe_rounds.py compat 100 > $OUT/rounds.log 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
echo done
