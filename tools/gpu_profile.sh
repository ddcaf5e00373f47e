#!/bin/bash
# Bench + rocprofv3 kernel-trace stats + HBM PMC passes (run on the GPU box via gpurun).
# usage: tools/gpu_profile.sh <tag> <schedule> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
SCHED=${1:-parallel}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 400 python3 bench.py --schedule "$SCHED" "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --schedule "$SCHED" --only --no-cpu-baseline --steps 200 --warmup 50 "$@" > "$OUT/trace.log" 2>&1 || { echo "trace failed $?"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C -T -d "$OUT/pmc_$C" -o run --output-format csv -- \
      python3 bench.py --schedule "$SCHED" --only --no-cpu-baseline --steps 100 --warmup 20 "$@" > "$OUT/pmc_$C.log" 2>&1 || { echo "pmc $C failed $?"; exit 1; }
done
find "$OUT" -name "*stats*.csv" | head
echo done
