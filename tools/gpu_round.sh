#!/bin/bash
# One GPU-box pass: the -m gpu suite, the default bench line, then the TransR
# transRNorm chain counters (KB2E_RPAR_STATS) on the headline config.
# usage (via gpurun): bash tools/gpu_round.sh <tag> [pytest-args...]
set -o pipefail
TAG=${1:-r10}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
(while sleep 45; do date >> "$OUT/heartbeat"; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 "$@" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed $?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -20 "$OUT/pytest.log"
timeout -k 10 500 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 --seed-epochs 5 > "$OUT/bench_stats.json" 2> "$OUT/bench_stats.err" || { echo "bench stats failed $?"; exit 1; }
grep "rpar_cons chunk" "$OUT/bench_stats.err" | tail -2
