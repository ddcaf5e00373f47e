#!/bin/bash
# The whole GPU suite (as the driver runs it), then the K5 and default bench lines.
set -o pipefail
OUT=gpurun_out/${1:-full}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed $?"; grep -E "^FAILED|Error|assert" $OUT/gpu_tests.log | head -20; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python -u bench.py --config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > $OUT/k5_bench.json 2> $OUT/k5_bench.err || { echo "k5 bench failed $?"; tail -5 $OUT/k5_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/k5_bench.json'));print('K5',d['value'],d['ms_per_step'],d['roofline']['kernels_avg_us'])"
