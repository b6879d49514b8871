#!/bin/bash
# HBM traffic (and MFMA activity) of the two roofline kernels of bench.py, one rocprofv3 --pmc pass per
# counter group (kernel-trace only; never combined with sys/runtime traces):
#   FFN up-projection GEMM  -- benchmarks/gemm_probe.py (the kernel alone, 20 launches)
#   grouped weight gradient -- bench.py --eager (one cfm_wgrad_group launch per step)
# Writes OUTDIR/{gemm_ffn_up,wgrad_group}_pmc.json (benchmarks/pmc_to_json.py).
# usage: bash benchmarks/pmc_roofline.sh OUTDIR
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1")
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {   # tag counters cmd...
  local tag=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d /tmp/pmc_$tag -o run -- "$@" > /dev/null 2>&1
  cp "$(find /tmp/pmc_$tag -name '*counter_collection.csv' | head -1)" "$OUT/$tag.csv"
  rm -rf /tmp/pmc_$tag
}
GP="python3 $R/benchmarks/gemm_probe.py 20"
BE="python3 $R/bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline --no-optimizer"
run ffn_fetch FETCH_SIZE $GP
run ffn_write WRITE_SIZE $GP
run ffn_mfma "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" $GP
run wg_fetch FETCH_SIZE $BE
run wg_write WRITE_SIZE $BE
run wg_mfma "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" $BE
# algorithmic bytes per launch (bench.py's gemm_desc_bytes at L15): FFN up A + B + y + pre-activation; wgrad the
# sum over the 136 GEMMs of dY + X read once + dW / db written once
python3 $R/benchmarks/pmc_to_json.py "$OUT" ffn "gemm_pipe_kernel" "gemm_ffn_up_pmc.json" "$GP" 112549888
python3 $R/benchmarks/pmc_to_json.py "$OUT" wg "false, true, false, " "wgrad_group_pmc.json" "$BE" 6851823616
rm -f "$OUT"/*.csv
