#!/bin/bash
# summary of a tools/gpu_cons.sh run (local)
D=gpurun_out/$1
tail -1 $D/pytest.log
grep -E "rpar_cons|rounds of" $D/rounds.log | tail -3
python3 - "$D" <<'PY'
import csv, json, sys
d = sys.argv[1]
b = json.load(open(d + "/bench_wave.json"))
r = b["roofline"]
print("value", round(b["value"]), "ms/step", round(b["ms_per_step"], 4), "frac", round(r["frac"], 4), "apply us",
      round(r["kernel_avg_us"], 1), "epoch", b["schedules"]["parallel"]["epoch"])
for x in csv.DictReader(open(d + "/kernel_stats.csv")):
    if "transr" in x["Name"] or "rpar" in x["Name"]:
        print(" ", x["Name"].split("(")[0][:60], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1))
PY
