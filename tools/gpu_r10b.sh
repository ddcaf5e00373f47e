set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r10b
timeout -k 10 900 python -u -m pytest tests/test_gpu_transr.py tests/test_gpu_parallel.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r10b/pytest.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/r10b/pytest.log; exit 1; }
tail -3 gpurun_out/r10b/pytest.log
for spec in "E 1000" "H 200" ; do set -- $spec; timeout -k 10 400 python tools/hits_parity.py --model $1 --epochs $2 --test 0 > gpurun_out/r10b/hits_$1.json 2> gpurun_out/r10b/hits_$1.err || exit 1; done
timeout -k 10 500 python tools/hits_parity.py --model R --epochs 100 --seed-epochs 500 --test 0 --compat 0 > gpurun_out/r10b/hits_R_fixed.json 2> gpurun_out/r10b/hits_R_fixed.err || exit 1
timeout -k 10 500 python tools/hits_parity.py --model R --epochs 100 --seed-epochs 500 --test 0 --compat 1 > gpurun_out/r10b/hits_R_compat.json 2> gpurun_out/r10b/hits_R_compat.err || exit 1
echo done
