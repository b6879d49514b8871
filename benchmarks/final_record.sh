#!/bin/bash
# The round's closing measurement record, part 1 (before the bench lines, which read it): one rocprofv3 kernel
# trace per benchmarked configuration of this build (-> summarize_trace.py family figures, lib md5 bound), then the
# PMC passes of the roofline kernels (separate --pmc runs, kernel trace only).  Each step under its own limit; the
# session stops at the first abort / timeout.
# usage: bash benchmarks/final_record.sh OUTDIR
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1")
mkdir -p "$OUT"
LIB=$R/nn_conformer_for_speech_recognition_amd/libcfm.so
step() {   # name limit cmd
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" bash -c "$*" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  tail -n 2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT: $name rc=$rc"; exit $rc; fi
}
trace() {   # key steps warmup bench-args...
  local key=$1 st=$2 wu=$3; shift 3
  step "trace_$key" 600 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/trace_$key -o run -- python3 $R/bench.py --steps $st --warmup $wu --no-cpu-baseline $* \
    > $OUT/trace_bench_$key.json && python3 $R/profiles/summarize_trace.py \
    \$(find $OUT/trace_$key -name '*kernel_trace.csv' | head -1) $OUT/trace_$key.json --config '$key' --warmup $wu \
    --steps $st --lib $LIB > $OUT/trace_summary_$key.txt && python3 $R/profiles/summarize.py \
    \$(find $OUT/trace_$key -name '*kernel_stats.csv' | head -1) auto 45 > $OUT/kernel_summary_$key.txt"
}
trace L15 10 3 --config L15
trace S15 10 3 --config S15
trace M15+specaug 10 3 --config M15 --specaug
trace L60 6 2 --config L60
trace L60+fp8 6 2 --config L60 --fp8
step pmc_roofline 900 "bash $R/benchmarks/pmc_roofline.sh $OUT/pmc"
step pmc_dgemm 900 "bash $R/benchmarks/pmc_dgemm.sh $OUT/pmc 5"
step pmc_fp8 600 "bash $R/benchmarks/pmc_fp8.sh $OUT/pmc 60186624"
echo "=== record done"
