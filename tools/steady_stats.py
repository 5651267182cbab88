"""Steady-state per-kernel statistics from a rocprofv3 --kernel-trace csv: the engine's kernels (fw::) after the
first `skip` launches of each (the warm-up's cold launches: first touches of the pane columns, code-object load),
with the median beside the mean.  Usage: python tools/steady_stats.py trace.csv out.csv [skip]"""
import collections
import csv
import statistics
import sys

path, out = sys.argv[1], sys.argv[2]
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 8
by = collections.defaultdict(list)
rows = []
for r in csv.DictReader(open(path)):
    if "fw::" in r["Kernel_Name"]:
        rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))))
rows.sort()
for _, name, d in rows:
    by[name].append(d)
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "Skipped", "AverageNs", "MedianNs", "MinNs", "MaxNs", "MaxOverMean"])
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        s = v[skip:] if len(v) > skip else v
        mean = sum(s) / len(s)
        w.writerow([name, len(s), len(v) - len(s), f"{mean:.1f}", f"{statistics.median(s):.1f}", min(s), max(s),
                    f"{max(s) / mean:.2f}"])
print(open(out).read())
