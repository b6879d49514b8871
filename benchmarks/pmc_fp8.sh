#!/bin/bash
# HBM traffic of the MX fp8 forward GEMM family (bench.py --config L60 --fp8's roofline_fp8): separate rocprofv3
# --pmc passes (FETCH_SIZE / WRITE_SIZE / MFMA counters) over one eager L60 fp8 step, the fp8 GEMM dispatches
# (gemm_pipe_kernel<..., GA false, GROUP false, F8 true, ...>) averaged per dispatch -> OUTDIR/gemm_fp8_pmc.json.
# usage: bash benchmarks/pmc_fp8.sh OUTDIR ALGORITHMIC_BYTES_PER_LAUNCH
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1"); ALG=$2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {   # tag counters cmd...
  local tag=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d /tmp/pmc_$tag -o run -- "$@" > /dev/null 2>&1
  cp "$(find /tmp/pmc_$tag -name '*counter_collection.csv' | head -1)" "$OUT/$tag.csv"
  rm -rf /tmp/pmc_$tag
}
BE="python3 $R/bench.py --config L60 --fp8 --eager --steps 1 --warmup 1 --no-cpu-baseline --no-optimizer"
run f8_fetch FETCH_SIZE $BE
run f8_write WRITE_SIZE $BE
run f8_mfma "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" $BE
PMC_AGG=mean PMC_SHAPE="11984,512,2048,17" python3 $R/benchmarks/pmc_to_json.py "$OUT" f8 "false, false, true, 128" \
  "gemm_fp8_pmc.json" "$BE" "$ALG"
rm -f "$OUT"/*.csv
