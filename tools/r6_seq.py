"""Durations (us) of each launch of the named kernels in order, from a rocprofv3 kernel trace csv.
Usage: python tools/r6_seq.py trace.csv name1,name2"""
import csv
import sys
names = sys.argv[2].split(",")
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in names:
        if f"::{k}" in n:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
rows.sort()
t0 = rows[0][0] if rows else 0
for s, e, k in rows:
    print(f"{(s - t0) / 1e3:10.1f} {k:18s} {(e - s) / 1e3:8.1f}")
