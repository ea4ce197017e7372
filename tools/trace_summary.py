"""Median per-launch time of the assignment kernels in a rocprofv3 kernel
trace (steady state = launches after the first three)."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = {}
for r in rows:
    n = r["Kernel_Name"].split("<")[0].split("(")[0]
    if n.startswith(("k_screen", "k_recheck", "k_label_sums")):
        by.setdefault(n, []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(sys.argv[2], " ".join("%s med %.3f ms (n=%d)" % (
    k, statistics.median(v[3:] or v), len(v)) for k, v in sorted(by.items())))
