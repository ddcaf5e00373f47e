set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 150 --timeout-method thread > gpurun_out/t/dist.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t/dist.log; exit 1; }
tail -3 gpurun_out/t/dist.log
