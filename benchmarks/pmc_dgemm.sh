#!/bin/bash
# PMC record of the d-wide GEMM family (benchmarks/dgemm_family.py --loop), one rocprofv3 --pmc pass per counter
# group (kernel-trace only; never combined with sys/runtime traces), each under its own time limit.
# usage: bash benchmarks/pmc_dgemm.sh OUTDIR [LOOPS]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1"); N=${2:-5}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {   # tag counters
  local tag=$1 ctr=$2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d /tmp/pmcd_$tag -o run -- \
    python3 $R/benchmarks/dgemm_family.py --loop $N > /dev/null 2>&1
  cp "$(find /tmp/pmcd_$tag -name '*counter_collection.csv' | head -1)" "$OUT/dg_$tag.csv"
  rm -rf /tmp/pmcd_$tag
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sqa "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
run sqb "SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum"
python3 $R/benchmarks/pmc_dgemm_json.py "$OUT" "python3 benchmarks/dgemm_family.py --loop $N"
rm -f "$OUT"/dg_*.csv
