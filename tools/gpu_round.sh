#!/bin/bash
# One GPU-box pass: the -m gpu suite, the default bench line, then a profile
# (rocprofv3 kernel stats + PMC) of the headline config.
# usage (via gpurun): bash tools/gpu_round.sh <tag> [pytest-args...]
set -o pipefail
TAG=${1:-r10}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed $?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 500 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
