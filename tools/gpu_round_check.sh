set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 300 python bench.py --config transr_fb15k > gpurun_out/r2/bench_transr.json 2> gpurun_out/r2/bench_transr.err && \
timeout -k 10 300 python bench.py --config transh_fb15k > gpurun_out/r2/bench_transh.json 2> gpurun_out/r2/bench_transh.err && \
timeout -k 10 300 python tools/hits_parity.py --model E --epochs 1000 --test 5000 > gpurun_out/r2/hits_E.json 2> gpurun_out/r2/hits_E.err && \
timeout -k 10 300 python tools/hits_parity.py --model H --epochs 200 --test 5000 > gpurun_out/r2/hits_H.json 2> gpurun_out/r2/hits_H.err && \
timeout -k 10 400 python tools/hits_parity.py --model R --epochs 100 --seed-epochs 200 --test 5000 > gpurun_out/r2/hits_R.json 2> gpurun_out/r2/hits_R.err
echo "exit $?"
