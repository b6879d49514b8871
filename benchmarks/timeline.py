"""Busy/idle analysis of a rocprofv3 --kernel-trace CSV: per step (delimited by conv1_fwd launches),
the wall span, the union of kernel intervals (GPU busy), and per-queue sums.
    python benchmarks/timeline.py kernel_trace.csv [n_last_steps]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")),
              r["Kernel_Name"]) for r in rows))
marks = [s for s, e, q, n in ks if "conv1_fwd" in n]
for i in range(max(0, len(marks) - 1 - nlast), len(marks) - 1):
    a, b = marks[i], marks[i + 1]
    seg = [(s, e, q, n) for s, e, q, n in ks if a <= s < b]
    busy, cur_s, cur_e = 0, None, None
    for s, e, q, n in seg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    perq = defaultdict(int)
    for s, e, q, n in seg:
        perq[q] += e - s
    gaps = sorted(((seg[j + 1][0] - max(x[1] for x in seg[:j + 1]), seg[j][3][:60]) for j in range(len(seg) - 1)),
                  reverse=True)[:8]
    print(f"step {i}: wall {(b-a)/1e6:.2f} ms, busy {busy/1e6:.2f} ms ({100*busy/(b-a):.1f}%), kernels {len(seg)}, "
          f"per-queue sum " + ", ".join(f"{q}:{v/1e6:.2f}" for q, v in perq.items()))
    for g, n in gaps:
        if g > 20000:
            print(f"    gap {g/1e3:7.1f} us after {n}")
