#!/bin/bash
# rel-pos attention changes: parity tests, kernel timing at L60, L60 bench line
set -o pipefail
O=$(pwd)/gpurun_out/rel_check; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_conformer.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
bash benchmarks/prof_bench_cmd.sh $O/stats.csv python3 $(pwd)/benchmarks/attn_rel_probe.py 3 && python3 profiles/summarize.py $O/stats.csv 4 6 && \
timeout -k 10 300 python bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_L60.json 2> $O/bench.err && python3 -c "import json;d=json.load(open('$O/bench_L60.json'));print('L60',d['ms_per_step'],d['value'],d['loss'],d['valid'])"
