#!/bin/bash
# 100-batch bench of one config under settings of one env var: tools/gpu_ab_cfg.sh TAG CONFIG VAR V1 V2 ... (V "-" = unset)
set -o pipefail
TAG=$1; CFG=$2; VAR=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for V in "$@"; do
  if [ "$V" = "-" ]; then unset $VAR; else export $VAR=$V; fi
  timeout -k 10 300 python bench.py --config $CFG --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/b_$V.json 2> $OUT/b_$V.err || { echo "bench $V failed"; tail $OUT/b_$V.err; exit 1; }
  echo "$CFG $VAR=$V: $(python3 -c "import json;d=json.load(open('$OUT/b_$V.json'));print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), 'epoch', round(d['schedules']['parallel']['epoch']['value']/1e6,3), d['roofline']['kernels_avg_us'])")"
done
