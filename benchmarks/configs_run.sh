#!/bin/bash
# One bench line per BASELINE.json config that fits one GPU (+ optional PMC roofline passes), into OUTDIR.
# usage: bash benchmarks/configs_run.sh OUTDIR [pmc]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$(realpath -m "$1"); mkdir -p "$O"
cd "$R"
b() {   # tag args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$O/bench_$tag.json" 2> "$O/bench_$tag.err" || { echo "bench $tag failed rc=$?"; tail -20 "$O/bench_$tag.err"; exit 1; }
  echo "== $tag"; python -c "import json,sys; r=json.load(open('$O/bench_$tag.json')); print(r['value'], r['ms_per_step'], r.get('dtype'))"
}
b L15 --steps 20 --warmup 5
b L60 --config L60 --steps 10 --warmup 3
b L60fp8 --config L60 --fp8 --steps 10 --warmup 3 --no-cpu-baseline
b S15 --config S15 --steps 20 --warmup 5 --no-cpu-baseline
b M15sa --config M15 --specaug --steps 20 --warmup 5 --no-cpu-baseline
b NST --nst --steps 20 --warmup 3
if [ "$2" = "pmc" ]; then
  bash benchmarks/pmc_roofline.sh "$O" || { echo "pmc failed"; exit 1; }
fi
