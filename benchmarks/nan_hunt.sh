#!/bin/bash
# NaN hunt driver for one gpurun call: every scenario under its own time limit; exit 1 (= NaN found) lets the
# chain continue, anything else (fault, abort, timeout) stops it.
set -u
OUT=${OUT:-gpurun_out/nan5}
mkdir -p "$OUT"
run() {
  local tag=$1; shift
  echo "=== $tag: $*" | tee -a "$OUT/summary.txt"
  timeout -k 10 240 "$@" > "$OUT/$tag.log" 2>&1
  local rc=$?
  grep '"summary"' "$OUT/$tag.log" >> "$OUT/summary.txt" || tail -3 "$OUT/$tag.log" >> "$OUT/summary.txt"
  echo "rc=$rc" >> "$OUT/summary.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
for sc in "$@"; do
  case $sc in
    L15g)   run L15g python -u benchmarks/nan_hunt.py --config L15 --probe --steps 12 ;;
    L15gp)  run L15gp python -u benchmarks/nan_hunt.py --config L15 --probe --poison --steps 8 ;;
    L15ep)  CFM_NANCHECK=1 run L15ep python -u benchmarks/nan_hunt.py --config L15 --eager --poison --steps 3 ;;
    S15g)   run S15g python -u benchmarks/nan_hunt.py --config S15 --probe --steps 12 ;;
    S15gp)  run S15gp python -u benchmarks/nan_hunt.py --config S15 --probe --poison --steps 8 ;;
    S15ep)  CFM_NANCHECK=1 run S15ep python -u benchmarks/nan_hunt.py --config S15 --eager --poison --steps 3 ;;
    L60g)   run L60g python -u benchmarks/nan_hunt.py --config L60 --probe --steps 10 ;;
    L60gp)  run L60gp python -u benchmarks/nan_hunt.py --config L60 --probe --poison --steps 6 ;;
    L15gn)  run L15gn python -u benchmarks/nan_hunt.py --config L15 --steps 6 ;;
    L15gd)  run L15gd python -u benchmarks/nan_hunt.py --config L15 --probe --steps 3 ;;
    S15gnp) run S15gnp python -u benchmarks/nan_hunt.py --config S15 --poison --steps 6 ;;
    S15gpd) run S15gpd python -u benchmarks/nan_hunt.py --config S15 --probe --poison --steps 3 ;;
    bench)  run bench python -u bench.py --no-cpu-baseline ;;
  esac
done
cat "$OUT/summary.txt"
