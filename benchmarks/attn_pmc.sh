#!/bin/bash
# PMC record of the L15 attention kernels: HBM traffic (FETCH_SIZE / WRITE_SIZE, one pass each) and the
# SQ instruction / wait / MFMA-busy groups (benchmarks/pmc_kernels.sh), every pass its own rocprofv3 run.
#   usage: bash benchmarks/attn_pmc.sh OUTDIR
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1")
mkdir -p "$OUT"
P="python3 $R/benchmarks/attn_pmc_probe.py 5"
bash "$R/benchmarks/pmc_kernels.sh" "$OUT/sq" $P > "$OUT/sq.txt"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d /tmp/ap_$c -o run -- $P > /dev/null 2>&1
  cp "$(find /tmp/ap_$c -name '*counter_collection.csv' | head -1)" "$OUT/$c.csv"
  rm -rf /tmp/ap_$c
done
python3 - "$OUT" <<'PY' > "$OUT/traffic.txt"
import csv, statistics, sys
by = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for r in csv.DictReader(open(f"{sys.argv[1]}/{c}.csv")):
        by.setdefault(r["Kernel_Name"][:60], {}).setdefault(c, []).append(float(r["Counter_Value"]))
print("kernel | fetch MB (x2 gfx950 correction) | write MB (medians per dispatch)")
for k, cs in by.items():
    f = statistics.median(cs.get("FETCH_SIZE", [0])) * 2 * 1024 / 1e6
    w = statistics.median(cs.get("WRITE_SIZE", [0])) * 1024 / 1e6
    print(f"{k} | {f:.1f} | {w:.1f}")
PY
rm -f "$OUT"/*.csv
cat "$OUT/traffic.txt" "$OUT/sq.txt"
