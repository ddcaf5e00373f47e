#!/bin/bash
# TransR n = 100 compat seed envelope (FB15k-shaped, 40 epochs, 500-epoch TransE
# seed, all 59,071 test triples), ORDERED (= the reference) and PARALLEL per
# glibc seed.  usage: tools/gpu_envelope_n100.sh <tag> <seeds, e.g. 7,8>
set -o pipefail
OUT=gpurun_out/${1:-env_n100}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1150 python -u tools/seed_envelope.py --model R --dim 100 --compat 1 --epochs 40 --seed-epochs 500 \
    --seeds ${2:-7} --out $OUT/envelope.jsonl > $OUT/envelope.log 2>&1 || { echo "envelope failed $?"; tail -5 $OUT/envelope.log; exit 1; }
tail -3 $OUT/envelope.log
