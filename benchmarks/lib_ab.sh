#!/bin/bash
# Same-box A/B of two builds of libcfm (CFM_LIB): attention probe at L15 + the L15 bench, interleaved.
# usage: bash benchmarks/lib_ab.sh BASE_SO [ROUNDS]
BASE=$1; R=${2:-2}
for r in $(seq 1 $R); do
  for lib in "$BASE" ""; do
    tag=${lib:-new}
    CFM_LIB=$lib timeout -k 10 300 python -u benchmarks/attn_probe.py 2>/dev/null | grep '^ATTN' | sed "s|^|[$tag] |" || exit 1
    out=$(CFM_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null) || { echo "bench failed: $tag"; exit 1; }
    echo "[$tag] L15 ms/step $(echo "$out" | grep '^{' | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
