#!/bin/bash
# One GPU pass for the folded front-end + DMA-staged attention forward: their parity tests, attention timings
# (DMA vs register staging), bench A/B (fold vs CFM_FFOLD=0) and a kernel summary.
set -o pipefail
O=gpurun_out/ff1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_frontfold.py tests/test_gpu_frontend.py tests/test_gpu_attention.py tests/test_gpu_conformer.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python benchmarks/attn_shapes.py > $O/attn_shapes.txt 2>&1 || { echo attn_shapes failed; tail $O/attn_shapes.txt; exit 1; }
grep libcfm $O/attn_shapes.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python -c "import json; r=json.load(open('$O/bench.json')); print('fold', r['value'], r['ms_per_step'], r['loss'], r['nonfinite_steps'])"
CFM_FFOLD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nofold.json 2> $O/bench_nofold.err || { echo bench2 failed; exit 1; }
python -c "import json; r=json.load(open('$O/bench_nofold.json')); print('nofold', r['value'], r['ms_per_step'], r['loss'])"
bash benchmarks/prof_bench.sh $O/kernel_stats.csv --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 && python profiles/summarize.py $O/kernel_stats.csv auto 60 > $O/kernel_summary.txt; head -30 $O/kernel_summary.txt
