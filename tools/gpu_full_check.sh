#!/bin/bash
# Round-end rehearsal on one MI355X: the whole -m gpu suite, smoke(), the default bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/full/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/full/gputests.log; exit 1; }
tail -3 gpurun_out/full/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/full/smoke.log; exit 1; }
cat gpurun_out/full/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || { echo "bench failed"; tail -20 gpurun_out/full/bench.err; exit 1; }
cut -c1-300 gpurun_out/full/bench.json
