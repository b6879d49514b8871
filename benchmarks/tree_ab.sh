#!/bin/bash
# Same-box A/B of two trees: BASE_DIR (a copy of bench.py + the package + its built libcfm.so) vs this tree,
# bench.py configs interleaved.  usage: bash benchmarks/tree_ab.sh BASE_DIR ROUNDS CONFIG...
R0=$(cd "$(dirname "$0")/.." && pwd)
BASE=$(realpath "$1"); R=$2; shift 2
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    for dir in "$BASE" "$R0"; do
      tag=$([ "$dir" = "$R0" ] && echo new || echo base)
      out=$(cd "$dir" && timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null) || { echo "bench failed: $tag $cfg"; exit 1; }
      echo "[$tag] $cfg ms/step $(echo "$out" | grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "nonfinite", d.get("nonfinite_steps"), "valid", d.get("valid"))')"
    done
  done
done
