set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
for c in transe_fb15k transr_fb15k; do
timeout -k 10 120 python bench.py --config $c --steps 300 --warmup 100 --only --no-cpu-baseline > gpurun_out/t/b.json || exit 1
python -c "import json; d=json.loads(open('gpurun_out/t/b.json').read().strip().splitlines()[-1]); print('$c', round(d['value']/1e6,2), d['roofline']['kernels_avg_us'], d['roofline']['frac'])"
done
