#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench line, rocprofv3 --stats summary.
# usage: bash benchmarks/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
bash benchmarks/prof_bench.sh $O/kernel_stats.csv --steps 5 --warmup 2 --no-cpu-baseline || { echo "prof failed"; tail -20 $O/kernel_stats.log; exit 1; }
python profiles/summarize.py $O/kernel_stats.csv auto 40 > $O/kernel_summary.txt
head -45 $O/kernel_summary.txt
