set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r10d
timeout -k 10 600 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_cli.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r10d/pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r10d/pytest.log; exit 1; }
tail -3 gpurun_out/r10d/pytest.log
