#!/bin/bash
# rocprofv3 --pmc passes (one counter group per run, kernel-trace only) over a probe command; prints the
# per-kernel median of each counter.   usage: bash benchmarks/pmc_kernels.sh OUTDIR cmd...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pk_$i -o run -- "$@" > /dev/null 2>&1 || echo "FAILED $grp"
  f=$(find /tmp/pk_$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/pass$i.csv"
  rm -rf /tmp/pk_$i
done
python3 - "$OUT" <<'PY'
import csv, glob, statistics, sys
by = {}
for f in sorted(glob.glob(sys.argv[1] + "/pass*.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        by.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, cs in by.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {statistics.median(v):16.0f}")
    if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:   # gfx950: FETCH_SIZE counts half of 16-B/lane streaming reads
        fb = 2 * 1024 * statistics.median(cs.get("FETCH_SIZE", [0]))
        wb = 1024 * statistics.median(cs.get("WRITE_SIZE", [0]))
        print(f"    {'HBM read MB (2*FETCH_SIZE)':28s} {fb / 1e6:16.1f}\n    {'HBM write MB (WRITE_SIZE)':28s} {wb / 1e6:16.1f}")
    if "TCC_HIT_sum" in cs:
        h, m = statistics.median(cs["TCC_HIT_sum"]), statistics.median(cs.get("TCC_MISS_sum", [0]))
        print(f"    {'L2 hit rate':28s} {h / max(h + m, 1):16.3f}")
PY
