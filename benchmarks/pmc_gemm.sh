#!/bin/bash
# PMC passes over benchmarks/gemm_probe.py for the GEMM kernel variants (one counter group per
# rocprofv3 run; kernel-trace only, never combined with sys/runtime traces).
# usage: bash benchmarks/pmc_gemm.sh OUTDIR "MODES" [--plain]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1"); MODES=$2; EXTRA=$3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for m in $MODES; do
  for grp in "SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM" \
             "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" "FETCH_SIZE" "WRITE_SIZE"; do
    tag=$(echo $grp | tr ' ' '_')
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc_${m}_${tag} -o run -- \
      python3 $R/benchmarks/gemm_probe.py 10 --mode $m $EXTRA > /dev/null 2>&1 || echo "FAILED $m $grp"
    f=$(find /tmp/pmc_${m}_${tag} -name "*counter_collection.csv" | head -1)
    [ -n "$f" ] && python3 $R/benchmarks/pmc_summarize.py "$f" >> "$OUT/pmc_mode$m.txt"
    rm -rf /tmp/pmc_${m}_${tag}
  done
done
