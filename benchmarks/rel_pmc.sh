#!/bin/bash
# rel-pos attention at the L60 shape: timing with / without attention dropout, then PMC passes
set -o pipefail
O=$(pwd)/gpurun_out/rel_pmc; mkdir -p $O
timeout -k 10 120 python3 benchmarks/attn_rel_probe.py 5 > $O/t_p01.txt 2>&1 && cat $O/t_p01.txt && \
timeout -k 10 120 python3 benchmarks/attn_rel_probe.py 5 --p 0 > $O/t_p0.txt 2>&1 && cat $O/t_p0.txt && \
bash benchmarks/prof_bench_cmd.sh $O/stats_p01.csv python3 $(pwd)/benchmarks/attn_rel_probe.py 3 && \
python3 profiles/summarize.py $O/stats_p01.csv 4 8 && \
bash benchmarks/prof_bench_cmd.sh $O/stats_p0.csv python3 $(pwd)/benchmarks/attn_rel_probe.py 3 --p 0 && \
python3 profiles/summarize.py $O/stats_p0.csv 4 8 && \
timeout -k 10 600 bash benchmarks/pmc_kernels.sh $O/pmc python3 $(pwd)/benchmarks/attn_rel_probe.py 2 > $O/pmc.txt 2>&1; cat $O/pmc.txt
