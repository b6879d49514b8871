#!/bin/bash
set -o pipefail
timeout -k 10 120 python3 benchmarks/v96_check.py || exit 1
timeout -k 10 120 python3 benchmarks/gemm_shapes.py --reps 3 --mode 3 | head -6 | sed 's/^/A /' && timeout -k 10 120 python3 benchmarks/gemm_shapes.py --reps 3 --mode 262147 | head -6 | sed 's/^/B /' || exit 1
for r in 1 2; do for m in 3 262147; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --gemm-mode $m 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('L15 mode $m', d['ms_per_step'], d['loss'])" || exit 1
done; done
