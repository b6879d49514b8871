#!/bin/bash
# rocprofv3 kernel-trace --stats of an arbitrary command; copies the stats CSV to OUT.
# usage: bash benchmarks/prof_bench_cmd.sh OUT.csv cmd args...
set -e
OUT=$(realpath -m "$1"); shift
D=/tmp/profc_$$
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- "$@" > "${OUT%.csv}.log" 2>&1
cp "$(find $D -name '*kernel_stats.csv' | head -1)" "$OUT"
rm -rf $D
