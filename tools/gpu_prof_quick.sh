#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pq
export TMPDIR=/tmp
(while sleep 45; do date >> gpurun_out/pq/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/pq/trace -o run --output-format csv -- python3 bench.py --only --no-cpu-baseline --no-epoch --late-epoch 0 --steps 100 --warmup 100 --seed-epochs 5 > gpurun_out/pq/trace.log 2>&1 || { echo "trace failed $?"; tail -5 gpurun_out/pq/trace.log; exit 1; }
head -12 gpurun_out/pq/trace/run_kernel_stats.csv | cut -d, -f1-6
