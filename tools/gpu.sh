#!/bin/bash
# One entry point for the GPU-box runs (through gpurun); every step runs under its
# own time limit, steps are chained so that the first failure ends the call, and
# the logs land under gpurun_out/<tag>/.
#
#   bash tools/gpu.sh suite    <tag> [pytest args]          the -m gpu suite, one process
#   bash tools/gpu.sh tests    <tag> <pytest selection...>  selected GPU tests
#   bash tools/gpu.sh bench    <tag> [bench.py args]        one bench line (default: the driver's)
#   bash tools/gpu.sh ab       <tag> <config> <VAR> <v1> [v2 ...]   100-batch lines per env setting ("-" = unset)
#   bash tools/gpu.sh profile  <tag> <schedule> [bench args]  bench + rocprofv3 trace + HBM / f64-MFMA PMC passes
#   bash tools/gpu.sh envelope <tag> <model> <dim> <compat> <epochs> <seeds> [batches] [schedules] [sub-batches]
#   bash tools/gpu.sh hits     <tag>                        FB15k-shaped Hits@10 schedule parity, four configs
#   bash tools/gpu.sh k5       <tag>                        n > 64 parity tests, K5 tests, the K5 line
#   bash tools/gpu.sh final    <tag>                        suite + default line + K5 line
#   bash tools/gpu.sh k5stats  <tag> <chain> [chain ...]      K5 chain phase counters per KB2E_RPAR_CHAIN ("-" = unset;
#                                                           CFG=<config> for another bench config)
#   bash tools/gpu.sh timeline <tag>                        kernel timeline of the driver-style line (K=20)
#   bash tools/gpu.sh pmcw     <tag>                        TransH phase-B kernels' SQ counters (occupancy, LDS, waits)
# (ab: AB_EPOCH=1 also times the whole epoch and epoch 50, e.g. the TransH gate sweep
#  AB_EPOCH=1 bash tools/gpu.sh ab gate transh_fb15k KB2E_HPAR_ORTH_MIN 0 16 64 256)
set -o pipefail
CMD=$1; TAG=${2:-$1}; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
(while sleep 45; do date >> "$OUT/heartbeat"; done) &
HB=$!
trap "kill $HB" EXIT

fail() { echo "$1 failed ($2)"; [ -f "$3" ] && { grep -E "^FAILED|Error|assert" "$3" | head -20; tail -15 "$3"; }; exit 1; }
line() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline',{});print(sys.argv[2],d['value'],'ms/step',round(d['ms_per_step'],4),'frac',r.get('frac'),'traffic_frac',r.get('traffic_frac'),r.get('kernels_avg_us'))" "$1" "$2"; }
pytest_run() {  # <log> <limit> args...
  local log=$1 lim=$2; shift 2
  timeout -k 10 "$lim" python -u -m pytest -x -v --timeout 400 --timeout-method thread --durations=15 "$@" > "$log" 2>&1 || fail pytest $? "$log"
  tail -1 "$log"
}
bench_run() {  # <name> <limit> args...
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" python -u bench.py "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || fail "bench $n" $? "$OUT/$n.err"
  line "$OUT/$n.json" "$n"
}
K5="--config transr_k5 --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5"

case "$CMD" in
  suite) pytest_run "$OUT/pytest.log" 1100 tests -m gpu "$@" ;;
  tests) pytest_run "$OUT/pytest.log" 1100 "$@" ;;
  bench) bench_run bench 600 "$@" ;;
  ab)
    CFG=$1; VAR=$2; shift 2
    for V in "$@"; do
      if [ "$V" = "-" ]; then unset "$VAR"; else export "$VAR=$V"; fi
      if [ -n "$AB_EPOCH" ]; then EP="--late-epoch 50"; else EP="--no-epoch"; fi
      bench_run "ab_${V}" 400 --config "$CFG" --only --no-cpu-baseline $EP --steps 100 --warmup 100 || exit 1
    done ;;
  k5stats)  # the chain kernels' phase counters (KB2E_RPAR_STATS) on the K5 line, per KB2E_RPAR_CHAIN value
    for V in "$@"; do
      if [ "$V" = "-" ]; then unset KB2E_RPAR_CHAIN; else export KB2E_RPAR_CHAIN=$V; fi
      KB2E_RPAR_STATS=1 bench_run "st_$V" 300 --config "${CFG:-transr_k5}" --only --no-cpu-baseline --no-epoch --steps 10 --warmup 2 || exit 1
      grep "hot relations" "$OUT/st_$V.err" | tail -1 | sed 's/.*hot relations/hot/' | cut -c1-400
    done ;;
  timeline)
    timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl -o run --output-format csv -- \
        python3 bench.py --only --no-cpu-baseline --no-epoch --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || fail trace $? "$OUT/bench.log"
    python3 - "$(find /tmp/tl -name "*kernel_trace.csv" | head -1)" > "$OUT/timeline.txt" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[max(0, len(rows) - 400)]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kb2e::", "")[:56]
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} q{r.get('Queue_Id', '?'):>3} {n}")
PY
    tail -5 "$OUT/timeline.txt" ;;
  profile)
    SCHED=$1; shift
    bench_run bench 400 --schedule "$SCHED" "$@" || exit 1
    PASS="--schedule $SCHED --only --no-cpu-baseline --no-epoch --steps 100 --warmup 100"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
        python3 bench.py $PASS "$@" > "$OUT/trace.log" 2>&1 || fail trace $? "$OUT/trace.log"
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 400 rocprofv3 --pmc $C -T -d "$OUT/pmc_$C" -o run --output-format csv -- \
          python3 bench.py $PASS "$@" > "$OUT/pmc_$C.log" 2>&1 || fail "pmc $C" $? "$OUT/pmc_$C.log"
    done
    timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        -T -d "$OUT/pmc_MFMA" -o run --output-format csv -- \
        python3 bench.py $PASS "$@" > "$OUT/pmc_MFMA.log" 2>&1 || fail "pmc MFMA" $? "$OUT/pmc_MFMA.log"
    echo profile done ;;
  pmcw)  # TransH phase B split into its kernels (KB2E_HPAR_FUSE=0): SQ counters per kernel family
    export KB2E_HPAR_FUSE=0
    PASS="--config transh_fb15k --only --no-cpu-baseline --no-epoch --steps 100 --warmup 20"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
        python3 bench.py $PASS > "$OUT/trace.log" 2>&1 || fail trace $? "$OUT/trace.log"
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
        SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -T -d "$OUT/pmc_SQ" -o run --output-format csv -- \
        python3 bench.py $PASS > "$OUT/pmc_SQ.log" 2>&1 || fail "pmc SQ" $? "$OUT/pmc_SQ.log"
    python3 tools/pmc_table.py "$OUT/pmc_SQ/run_counter_collection.csv" > "$OUT/pmc_SQ.txt" && cat "$OUT/pmc_SQ.txt" ;;
  envelope)
    MODEL=$1; DIM=$2; COMPAT=$3; EP=$4; SEEDS=$5; NB=${6:-100}; SCH=${7:-ordered,parallel}; SUB=${8:-}
    timeout -k 10 1150 python -u tools/seed_envelope.py --model "$MODEL" --dim "$DIM" --compat "$COMPAT" --epochs "$EP" \
        --seed-epochs 500 --seeds "$SEEDS" --batches "$NB" --schedules "$SCH" ${SUB:+--sub $SUB} --out "$OUT/envelope.jsonl" \
        > "$OUT/envelope.log" 2>&1 || fail envelope $? "$OUT/envelope.log"
    grep "^seed" "$OUT/envelope.log" ;;
  hits)
    for a in "R_fixed --model R --dim 50 --epochs 100 --seed-epochs 500 --test 0 --compat 0" \
             "R_compat --model R --dim 50 --epochs 100 --seed-epochs 500 --test 0 --compat 1" \
             "H --model H --dim 100 --epochs 200 --test 0" "E --model E --dim 100 --epochs 1000 --test 0"; do
      set -- $a; n=$1; shift
      timeout -k 10 400 python -u tools/hits_parity.py "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || fail "hits $n" $? "$OUT/$n.err"
      echo "$n done"
    done ;;
  k5)
    pytest_run "$OUT/par.log" 400 tests/test_gpu_parallel.py -k "transr and (100 or 65 or 96 or 112 or 72 or 88 or 128)" || exit 1
    pytest_run "$OUT/k5t.log" 400 tests/test_gpu_k5.py || exit 1
    bench_run k5 400 $K5 ;;
  final)
    pytest_run "$OUT/pytest.log" 1000 tests -m gpu || exit 1
    bench_run default 600 || exit 1
    bench_run k5 400 $K5 ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
