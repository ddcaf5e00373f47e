#!/bin/bash
# FB15k-shaped Hits@10 schedule parity (PARALLEL vs ORDERED = reference) for all four
# configurations on the current kernels; JSON lines under gpurun_out/hp/.
set -o pipefail
mkdir -p gpurun_out/hp
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/hits_parity.py --model R --dim 50 --epochs 100 --seed-epochs 500 --test 0 --compat 0 > gpurun_out/hp/R_fixed.json 2> gpurun_out/hp/R_fixed.err && echo R_fixed done &&
timeout -k 10 400 python -u tools/hits_parity.py --model R --dim 50 --epochs 100 --seed-epochs 500 --test 0 --compat 1 > gpurun_out/hp/R_compat.json 2> gpurun_out/hp/R_compat.err && echo R_compat done &&
timeout -k 10 300 python -u tools/hits_parity.py --model H --dim 100 --epochs 200 --test 0 > gpurun_out/hp/H.json 2> gpurun_out/hp/H.err && echo H done &&
timeout -k 10 300 python -u tools/hits_parity.py --model E --dim 100 --epochs 1000 --test 0 > gpurun_out/hp/E.json 2> gpurun_out/hp/E.err && echo E done
