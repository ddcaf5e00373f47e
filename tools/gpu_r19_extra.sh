#!/bin/bash
# r19 evidence: FB15k-shaped Hits@10 schedule parity for TransH (200 epochs) and
# TransR compat on the current kernels, then the TransH PARALLEL profile.
set -o pipefail
mkdir -p gpurun_out/hp
export TMPDIR=/tmp
(while sleep 45; do date >> gpurun_out/hp/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u tools/hits_parity.py --model H --dim 100 --epochs 200 --test 0 > gpurun_out/hp/H.json 2> gpurun_out/hp/H.err && echo H done &&
timeout -k 10 400 python -u tools/hits_parity.py --model R --dim 50 --epochs 100 --seed-epochs 500 --test 0 --compat 1 > gpurun_out/hp/R_compat.json 2> gpurun_out/hp/R_compat.err && echo R_compat done &&
bash tools/gpu_profile.sh r19_transh_fb15k parallel --config transh_fb15k
