#!/bin/bash
# The -m gpu suite on the GPU box (one process, per-test timeout); log under gpurun_out/<tag>/.
set -o pipefail
TAG=${1:-suite}; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed $?"; grep -E "FAILED|Error|error" gpurun_out/$TAG/pytest.log | head -20; tail -60 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
