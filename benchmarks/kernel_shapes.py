"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace CSV over the last N steps
(steps delimited by conv1_fwd launches).
    python benchmarks/kernel_shapes.py kernel_trace.csv [n_last_steps] [name_filter]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 3
filt = sys.argv[3] if len(sys.argv) > 3 else ""
ks = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
marks = [int(r["Start_Timestamp"]) for r in ks if "conv1_fwd" in r["Kernel_Name"]]
lo = marks[max(0, len(marks) - 1 - nlast)]
hi = marks[-1]
agg = defaultdict(list)
for r in ks:
    s = int(r["Start_Timestamp"])
    if lo <= s < hi and filt in r["Kernel_Name"]:
        key = (r["Kernel_Name"][:90], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
        agg[key].append((int(r["End_Timestamp"]) - s) / 1e3)
tot = sum(sum(v) for v in agg.values())
print(f"{nlast} steps, {tot/1e3/nlast:.2f} ms/step of kernel time (filter {filt!r})")
for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:60]:
    print(f"{sum(v)/1e3/nlast:7.3f} ms/step  n/step={len(v)/nlast:6.1f}  avg={sum(v)/len(v):8.1f}us  "
          f"min={min(v):8.1f}  grid={key[1]}x{key[2]}x{key[3]} wg={key[4]}  {key[0]}")
