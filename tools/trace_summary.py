"""Summarise a rocprofv3 kernel trace: per-kernel count / total / average over
the last N launches of an anchor kernel's span, plus device idle time."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "apply"
last = int(sys.argv[3]) if len(sys.argv) > 3 else 300
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
sel = idx[-last:]
a, b = sel[0], sel[-1]
t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["End_Timestamp"])
print(f"span {(t1 - t0) / 1e3:.1f} us over {len(sel)} anchors: {(t1 - t0) / 1e3 / max(1, len(sel) - 1):.2f} us each")
busy, cnt = defaultdict(float), defaultdict(int)
for r in rows[a:b + 1]:
    n = r["Kernel_Name"].split("(")[0]
    n = n.replace("void ", "").replace("kb2e::", "")[:60]
    busy[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[n] += 1
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {k:60s} {cnt[k]:6d} {v:10.1f} us  avg {v / cnt[k]:8.2f}")
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[a:b + 1])
tot, (cs, ce) = 0, iv[0]
for s, e in iv[1:]:
    if s > ce:
        tot += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
tot += ce - cs
print(f"busy {tot / 1e3:.1f} us, idle {(t1 - t0 - tot) / 1e3:.1f} us")
