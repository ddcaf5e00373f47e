#!/bin/bash
# Bench + rocprofv3 kernel-trace stats + HBM PMC passes + an f64 MFMA PMC pass
# (run on the GPU box via gpurun), summarised by tools/summarize_profile.py.
# usage: tools/gpu_profile.sh <tag> <schedule> [bench args...]
# The trace and PMC passes run 100 warmup + 100 timed batches of the schedule
# (200 batches: summarize_profile.py's per-batch divisor).
set -o pipefail
TAG=${1:-r01}; shift
SCHED=${1:-parallel}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
(while sleep 45; do date >> "$OUT/heartbeat"; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python3 bench.py --schedule "$SCHED" "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; exit 1; }
cat "$OUT/bench.json"
PASS="--schedule $SCHED --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py $PASS "$@" > "$OUT/trace.log" 2>&1 || { echo "trace failed $?"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C -T -d "$OUT/pmc_$C" -o run --output-format csv -- \
      python3 bench.py $PASS "$@" > "$OUT/pmc_$C.log" 2>&1 || { echo "pmc $C failed $?"; exit 1; }
done
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -T -d "$OUT/pmc_MFMA" -o run --output-format csv -- \
    python3 bench.py $PASS "$@" > "$OUT/pmc_MFMA.log" 2>&1 || { echo "pmc MFMA failed $?"; exit 1; }
find "$OUT" -name "*stats*.csv" | head
echo done
