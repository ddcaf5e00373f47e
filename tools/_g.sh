set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest tests/test_gpu_cli.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t/cli.log 2>&1 || { echo "tests failed"; grep -E "^E |Error|assert" gpurun_out/t/cli.log | head -30; exit 1; }
tail -3 gpurun_out/t/cli.log
