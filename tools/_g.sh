set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t/prof -o run --output-format csv -- python3 bench.py --config transh_fb15k --only --no-cpu-baseline --steps 100 --warmup 300 > gpurun_out/t/prof.log 2>&1 || { echo "prof failed"; exit 1; }
cut -c1-200 gpurun_out/t/prof.log | grep metric
