#!/bin/bash
# Same-box A/B of two builds of libcfm (CFM_LIB) on bench.py configs, interleaved.
# usage: bash benchmarks/lib_ab_cfg.sh BASE_SO ROUNDS CONFIG...
BASE=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    for lib in "$BASE" ""; do
      tag=${lib:-new}
      out=$(CFM_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null) || { echo "bench failed: $tag $cfg"; exit 1; }
      echo "[$tag] $cfg ms/step $(echo "$out" | grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ctc", d.get("ctc_head", {}).get("ms"))')"
    done
  done
done
