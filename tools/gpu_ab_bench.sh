#!/bin/bash
# Driver-style bench (K=20, W=5) and the 100-step rate under settings of one env var:
# tools/gpu_ab_bench.sh TAG VAR V1 V2 ...  (V "-" = unset)
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for V in "$@"; do
  for S in 20 100; do
    if [ "$V" = "-" ]; then unset $VAR; else export $VAR=$V; fi
    timeout -k 10 300 python bench.py --only --no-cpu-baseline --no-epoch --steps $S --warmup 5 > $OUT/b_${V}_$S.json 2> $OUT/b_${V}_$S.err || { echo "bench $V $S failed"; tail $OUT/b_${V}_$S.err; exit 1; }
    echo "$VAR=$V steps $S: $(python3 -c "import json;d=json.load(open('$OUT/b_${V}_$S.json'));print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4))")"
  done
done
