"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
arg = sys.argv[2] if len(sys.argv) > 2 else "1"
if arg == "auto":
    # executed training steps = launches of the grouped weight-gradient kernel (one per step, eager warm-up,
    # timed replays and probe-graph replays alike)
    steps = sum(float(r["Calls"]) for r in rows if "gemm_pipe_kernel" in r["Name"] and "false, true, false, " in r["Name"])
else:
    steps = float(arg)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms over {steps:g} steps = {tot/1e6/steps:.2f} ms/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
          f"calls/step={float(r['Calls'])/steps:7.1f} avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
