"""Kernel timeline of a rocprofv3 --kernel-trace run (gpurun_out/prof_trace/run_kernel_trace.csv): per
kernel name the mean duration, and for the timed steps the gaps between consecutive launches and the
time two launches overlapped.  Usage: python tools/timeline.py [trace.csv] [first_kernel_index]"""
import csv
import sys
import collections

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_trace/run_kernel_trace.csv"
rows = []
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if "fw::" not in name:
        continue
    short = name.split("fw::")[1].split("<")[0].split("(")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
rows.sort()
skip = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 3
rows = rows[skip:]
dur = collections.defaultdict(list)
for s, e, n in rows:
    dur[n].append((e - s) / 1e3)
for n, v in sorted(dur.items()):
    print(f"{n:24s} n={len(v):4d} mean={sum(v)/len(v):8.2f} us  min={min(v):8.2f}  max={max(v):8.2f}")
busy = 0
cur_s, cur_e = rows[0][0], rows[0][1]
gaps = collections.defaultdict(list)
overlap = 0
prev = rows[0]
for s, e, n in rows[1:]:
    if s < prev[1]:
        overlap += min(e, prev[1]) - s
    else:
        gaps[(prev[2], n)].append((s - prev[1]) / 1e3)
    if s > cur_e:
        busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev = (s, e, n) if e > prev[1] else prev
busy += cur_e - cur_s
span = rows[-1][1] - rows[0][0]
print(f"span {span/1e3:.1f} us, busy {busy/1e3:.1f} us ({100*busy/span:.0f}%), overlap {overlap/1e3:.1f} us")
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
    print(f"gap {k[0]:>16s} -> {k[1]:16s} n={len(v):4d} mean={sum(v)/len(v):6.2f} us total={sum(v):8.1f}")
