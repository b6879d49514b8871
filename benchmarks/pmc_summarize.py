"""Median per-dispatch value of every counter in a rocprofv3 counter_collection.csv, for the
GEMM kernel dispatches only."""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "gemm" in r.get("Kernel_Name", "")]
by = {}
for r in rows:
    by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in sorted(by.items()):
    print(f"{k:28s} median {statistics.median(v):16.1f}  (n={len(v)})  kernel={rows[0]['Kernel_Name'][:60]}")
