#!/bin/bash
# L2 hit rate of the grouped weight-gradient launch (one --pmc pass) + the same for the FFN-up GEMM
R=$(pwd)
OUT=$R/gpurun_out/r05q; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/wgl2 -o run -- python3 $R/bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline --no-optimizer > $OUT/bench.log 2>&1
f=$(find /tmp/wgl2 -name '*counter_collection.csv' | head -1)
cp $f $OUT/l2.csv
python3 - $OUT/l2.csv <<'PY'
import csv, sys, collections
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    by[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(by.items(), key=lambda kv: -sum(kv[1].get("TCC_MISS_sum", [0]))):
    h, m = sum(cs.get("TCC_HIT_sum", [0])), sum(cs.get("TCC_MISS_sum", [0]))
    n = len(cs.get("TCC_HIT_sum", []))
    print(f"{h / max(h + m, 1):6.3f} hit  {m * 128 / 1e9 / max(n,1):8.3f} GB-miss(x128B)/launch  n={n:4d}  {k}")
PY
