#!/bin/bash
# Same-box A/B of bench.py variants selected by environment strings (interleaved, R rounds).
# usage: bash benchmarks/ab_bench.sh ROUNDS "ENV_A" "ENV_B" ...   (use "-" for no extra env)
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    e=$v; [ "$v" = "-" ] && e=""
    out=$(env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null) || { echo "bench failed: $v"; exit 1; }
    echo "round $r [$v] $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
