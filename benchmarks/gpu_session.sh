#!/bin/bash
# One GPU session on the box: steps chained so that a crash / timeout / abort ends the session (test failures do
# not).  usage: bash benchmarks/gpu_session.sh OUTDIR STEP...
#   steps: fulldepth | gputests | ktests | dgemm | wide | wgrad | attn | bench | benchL60 | dp | pmc_dgemm | ktrace | <any shell command in quotes>
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd "$R"
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" bash -c "$*" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  tail -n 3 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "ABORT: $name rc=$rc"; exit $rc; fi
  return 0
}
NC=0
for s in "$@"; do
  case $s in
    fulldepth) run fulldepth 900 "$PYT -s tests/test_gpu_fulldepth.py" ;;
    gputests) run gputests 900 "$PYT -q -m gpu tests --ignore=tests/test_gpu_fulldepth.py" ;;
    dgemm) run dgemm 300 "python -u benchmarks/dgemm_family.py && python -u benchmarks/dgemm_family.py --mode 524291" ;;
    wide) run wide 300 "python -u benchmarks/wide_gemm.py --modes 3" ;;
    wgrad) run wgrad 300 "python -u benchmarks/wgrad_modes.py --modes 3" ;;
    attn) run attn 300 "python -u benchmarks/attn_probe.py" ;;
    rel) run rel 300 "python -u benchmarks/rel_modes.py" ;;
    relprof) run relprof 600 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/relprof -o run -- python3 $R/benchmarks/rel_modes.py --reps 2 && python3 $R/profiles/summarize.py \$(find $OUT/relprof -name '*kernel_stats.csv' | head -1) 1 25 > $OUT/rel_kernel_summary.txt" ;;
    ktests) run ktests 900 "$PYT -q tests/test_gpu_kernels.py tests/test_gpu_attention.py tests/test_gpu_conformer.py tests/test_gpu_fulldepth.py tests/test_gpu_frontfold.py tests/test_gpu_graph.py" ;;
    bench) run bench 600 "python -u bench.py --gpus 1 --steps 20 --warmup 5" ;;
    benchL60) run benchL60 600 "python -u bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline" ;;
    dp) run dp 900 "for f in '' '--dp-overlap' '--dp-overlap --grad-bf16' '--dp-overlap --dp-chunk-layers 17' ''; do python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \$f || exit 1; done" ;;
    pmc_dgemm) run pmc_dgemm 900 "bash benchmarks/pmc_dgemm.sh $OUT 5" ;;
    ktrace) run ktrace 600 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline && python3 $R/profiles/summarize.py \$(find $OUT/ktrace -name '*kernel_stats.csv' | head -1) auto 45 > $OUT/kernel_summary.txt" ;;
    trace|trace:*)   # rocprofv3 kernel trace of a bench.py run -> profiles/summarize_trace.py family figures
      cfg=${s#trace}; cfg=${cfg#:}; cfg=${cfg:-L15}
      run trace_$cfg 600 "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$cfg -o run -- python3 $R/bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $OUT/trace_bench_$cfg.json && python3 $R/profiles/summarize_trace.py \$(find $OUT/trace_$cfg -name '*kernel_trace.csv' | head -1) $OUT/trace_$cfg.json --config $cfg --warmup 3 --steps 10 --lib $R/nn_conformer_for_speech_recognition_amd/libcfm.so > $OUT/trace_summary_$cfg.txt && python3 $R/profiles/summarize.py \$(find $OUT/trace_$cfg -name '*kernel_stats.csv' | head -1) auto 45 > $OUT/kernel_summary_$cfg.txt" ;;
    *) NC=$((NC + 1)); run custom$NC 900 "$s" ;;
  esac
done
echo "=== session done"
