#!/bin/bash
set -o pipefail
O=$(pwd)/gpurun_out/v96; mkdir -p $O
timeout -k 10 120 python3 benchmarks/v96_check.py || exit 1
timeout -k 10 120 python3 benchmarks/gemm_shapes.py --reps 3 --mode 3 > $O/A.txt 2>/dev/null && timeout -k 10 120 python3 benchmarks/gemm_shapes.py --reps 3 --mode 262147 > $O/B.txt 2>/dev/null || exit 1
sed -n 1,6p $O/A.txt | sed 's/^/A /'; sed -n 1,6p $O/B.txt | sed 's/^/B /'
for r in 1 2; do for m in 3 262147; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --gemm-mode $m > $O/b_$m.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$m.json')); print('L15 mode $m', d['ms_per_step'], d['loss'])"
done; done
