#!/bin/bash
# A/B of the tail-balanced GEMM row split (default) vs one launch (CFM_GEMM_MODE=131075): GEMM tests, bench
# lines (interleaved x2), kernel summary of the default
set -o pipefail
O=gpurun_out/split; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
for v in "-" "CFM_GEMM_MODE=131075"; do
  e=$v; [ "$v" = "-" ] && e=""
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b15.json 2>$O/b15.err || { echo "bench $v failed"; tail $O/b15.err; exit 1; }
  python -c "import json; r=json.load(open('$O/b15.json')); print('L15 [$v]', r['value'], r['ms_per_step'], r['loss'], r['nonfinite_steps'])"
done
done
bash benchmarks/prof_bench.sh $O/k15.csv --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 && python profiles/summarize.py $O/k15.csv auto 60 > $O/k15.txt; head -12 $O/k15.txt | cut -c1-140
