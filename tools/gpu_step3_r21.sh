#!/bin/bash
# TransH tests + profile at the gate's default, then the last n = 100 envelope seed.
set -o pipefail
mkdir -p gpurun_out/r21_step3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_transh.py -x -q --timeout 200 --timeout-method thread -k "transh" > gpurun_out/r21_step3/h.log 2>&1 || { echo "transh tests failed $?"; tail -5 gpurun_out/r21_step3/h.log; exit 1; }
tail -1 gpurun_out/r21_step3/h.log
bash tools/gpu_profile.sh r21_transh parallel --config transh_fb15k || exit 1
bash tools/gpu_envelope_n100.sh env_n100_r21c 11 || exit 1
