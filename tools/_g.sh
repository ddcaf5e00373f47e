set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest tests/test_gpu_parallel.py tests/test_gpu_transr.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t/par.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t/par.log; exit 1; }
tail -1 gpurun_out/t/par.log
timeout -k 10 120 python bench.py --config transr_fb15k --steps 300 --warmup 100 --only --no-cpu-baseline > gpurun_out/t/b.json || exit 1
python -c "import json; d=json.loads(open('gpurun_out/t/b.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), d['roofline']['kernels_avg_us'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t/prof -o run --output-format csv -- python3 bench.py --config transr_fb15k --only --no-cpu-baseline --steps 100 --warmup 20 > gpurun_out/t/prof.log 2>&1 || { echo "prof failed"; exit 1; }
