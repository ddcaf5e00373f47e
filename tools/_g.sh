set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 120 --timeout-method thread -k transr > gpurun_out/t/par.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t/par.log; exit 1; }
tail -1 gpurun_out/t/par.log
timeout -k 10 120 python tools/probe_rounds.py compat > gpurun_out/t/rounds.log 2>&1 || { echo "probe failed"; tail gpurun_out/t/rounds.log; exit 1; }
tail -4 gpurun_out/t/rounds.log
timeout -k 10 120 python bench.py --config transr_fb15k --steps 300 --warmup 100 --only --no-cpu-baseline > gpurun_out/t/b.json || exit 1
python -c "import json; d=json.loads(open('gpurun_out/t/b.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), d['roofline']['kernels_avg_us'], d['roofline']['frac'])"
