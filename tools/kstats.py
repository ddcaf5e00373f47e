"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (dev tool)."""
import csv
import glob
import sys

f = sys.argv[1] if len(sys.argv) > 1 else sorted(glob.glob("gpurun_out/t/prof/**/*kernel_stats.csv", recursive=True))[0]
for x in list(csv.DictReader(open(f)))[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    nm = x["Name"].replace("kb2e::RParArgs, kb2e::RParBufs<double>", "").replace("kb2e::", "")[:60]
    print(f"{nm:62s} {x['Calls']:>5s} {float(x['TotalDurationNs']) / 1e6:8.2f} ms {float(x['AverageNs']) / 1e3:8.1f} us {x['Percentage'][:5]}")
