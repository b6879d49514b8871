#!/bin/bash
# rocprofv3 kernel-trace --stats of a short bench.py run; copies only the stats CSV to OUT.
# usage: bash benchmarks/prof_bench.sh OUT.csv [bench.py args...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "$1"); shift
D=/tmp/prof_$$
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $R/bench.py "$@" \
  > "${OUT%.csv}.log" 2>&1
cp "$(find $D -name '*kernel_stats.csv' | head -1)" "$OUT"
rm -rf $D
