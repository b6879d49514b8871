"""Print the kernels around the largest idle gaps of a rocprofv3 kernel trace (last steps).
    python benchmarks/gap_context.py kernel_trace.csv [ngaps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ng = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")),
             r["Kernel_Name"][:70]) for r in rows)
ks = ks[len(ks) // 2:]
gaps = []
end = ks[0][1]
for i in range(1, len(ks)):
    if ks[i][0] > end:
        gaps.append((ks[i][0] - end, i))
    end = max(end, ks[i][1])
for g, i in sorted(gaps, reverse=True)[:ng]:
    print(f"gap {g/1e3:.1f} us")
    for j in range(max(0, i - 4), min(len(ks), i + 4)):
        s, e, q, n = ks[j]
        print(f"   {'>>' if j == i else '  '} q{q} {(e-s)/1e3:8.1f}us  {n}")
