#!/bin/bash
# transRNorm chain phase counters under timing-only KB2E_CONS_DBG switches (wrong results).
set -o pipefail
OUT=gpurun_out/${1:-cdbg}
mkdir -p $OUT
export TMPDIR=/tmp
for D in 0 1; do
  KB2E_CONS_DBG=$D KB2E_RPAR_STATS=1 timeout -k 10 300 python -u bench.py --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100 --seed-epochs 5 > $OUT/b$D.json 2> $OUT/b$D.err || exit 1
  echo "dbg=$D $(grep 'rpar_cons chunk phases' $OUT/b$D.err | tail -1 | sed 's/.*hot relations//')"
  python -c "import json;d=json.load(open('$OUT/b$D.json'));print(d['value'], d['roofline']['kernels_avg_us'])"
done
