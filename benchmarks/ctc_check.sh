#!/bin/bash
set -o pipefail
O=$(pwd)/gpurun_out/ctc_check; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ctc.py tests/test_gpu_nst.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
bash benchmarks/prof_bench.sh $O/stats.csv --config L60 --steps 4 --warmup 2 --no-cpu-baseline && python3 profiles/summarize.py $O/stats.csv auto 12 | grep -i "ctc\|total" && \
timeout -k 10 300 python bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_L60.json 2> $O/bench.err && python3 -c "import json;d=json.load(open('$O/bench_L60.json'));print('L60',d['ms_per_step'],d['value'],d['loss'],d['valid'])"
