set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r10e
timeout -k 10 120 rocprofv3 -L > gpurun_out/r10e/counters.txt 2>&1 || echo "list failed $?"
bash tools/gpu_profile.sh r10_transr_fb15k parallel --config transr_fb15k || exit 1
