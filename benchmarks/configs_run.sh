#!/bin/bash
# One bench line per BASELINE.json config that fits one GPU (+ the PMC roofline passes), into OUTDIR.
# usage: bash benchmarks/configs_run.sh OUTDIR [pmc]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$(realpath -m "$1"); mkdir -p "$O"
cd "$R"
b() {   # tag args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$O/bench_$tag.json" 2> "$O/bench_$tag.err" || { echo "bench $tag failed rc=$?"; tail -20 "$O/bench_$tag.err"; exit 1; }
  echo "== $tag"; cat "$O/bench_$tag.json"
}
b L15 --steps 20 --warmup 5
b L60 --config L60 --steps 10 --warmup 3
b S15 --config S15 --steps 20 --warmup 5 --no-cpu-baseline
b M15sa --config M15 --specaug --steps 20 --warmup 5 --no-cpu-baseline
if [ "$2" = "pmc" ]; then
  bash benchmarks/pmc_roofline.sh "$O" || { echo "pmc failed"; exit 1; }
  cat "$O"/*_pmc.json
fi
