#!/bin/bash
# TransH normOrth relation-pass gate: epoch-0 (100 batches), whole-epoch and
# epoch-50 figures for several KB2E_HPAR_ORTH_MIN thresholds.
set -o pipefail
OUT=gpurun_out/${1:-transh_gate}
mkdir -p $OUT
export TMPDIR=/tmp
for m in ${2:-0 16 64 256}; do
  KB2E_HPAR_ORTH_MIN=$m timeout -k 10 300 python -u bench.py --config transh_fb15k --only --no-cpu-baseline --steps 100 --warmup 100 > $OUT/h_$m.json 2> $OUT/h_$m.err || { echo "bench $m failed $?"; tail -5 $OUT/h_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/h_$m.json'));p=d['schedules']['parallel'];print('min',$m,d['value'],p['epoch']['value'] if p.get('epoch') else None,p['late_epoch']['value'] if p.get('late_epoch') else None,d['roofline']['frac'])"
done
