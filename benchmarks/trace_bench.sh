#!/bin/bash
# rocprofv3 --kernel-trace (no counters) of a short bench.py run -> timeline analysis.
# usage: bash benchmarks/trace_bench.sh OUTDIR [bench.py args...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1"); shift
mkdir -p $OUT
D=/tmp/trace_$$
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 $R/bench.py "$@" > $OUT/trace_bench.log 2>&1
cp "$(find $D -name '*kernel_trace.csv' | head -1)" $OUT/kernel_trace.csv
rm -rf $D
python3 $R/benchmarks/timeline.py $OUT/kernel_trace.csv 3 | tee $OUT/timeline.txt
