#!/bin/bash
# A/B of the precomputed attention-dropout bits (default) vs in-kernel hashing (CFM_DISABLE=dropmask):
# attention tests, L15 and L60 bench lines, per-kernel summary of each L15 variant.
set -o pipefail
O=gpurun_out/mask; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "-" "CFM_DISABLE=dropmask"; do
  e=$v; [ "$v" = "-" ] && e=""
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b15.json 2>$O/b15.err || { echo "bench $v failed"; tail $O/b15.err; exit 1; }
  python -c "import json; r=json.load(open('$O/b15.json')); print('L15 [$v]', r['value'], r['ms_per_step'], r['loss'], r['nonfinite_steps'])"
  env $e timeout -k 10 400 python bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline > $O/b60.json 2>$O/b60.err || { echo "bench60 $v failed"; tail $O/b60.err; exit 1; }
  python -c "import json; r=json.load(open('$O/b60.json')); print('L60 [$v]', r['value'], r['ms_per_step'], r['loss'], r['nonfinite_steps'])"
done
bash benchmarks/prof_bench.sh $O/k15.csv --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 && python profiles/summarize.py $O/k15.csv auto 60 > $O/k15.txt; grep -E "attn|ada_|total" $O/k15.txt | cut -c1-120
