#!/bin/bash
set -o pipefail
O=$(pwd)/gpurun_out/conv_pmc; mkdir -p $O
timeout -k 10 120 python3 benchmarks/conv_probe.py 20 && \
bash benchmarks/prof_bench_cmd.sh $O/stats.csv python3 $(pwd)/benchmarks/conv_probe.py 20 && python3 profiles/summarize.py $O/stats.csv 21 10 && \
timeout -k 10 600 bash benchmarks/pmc_kernels.sh $O/pmc python3 $(pwd)/benchmarks/conv_probe.py 3 > $O/pmc.txt 2>&1; grep -A15 "glu_dwconv" $O/pmc.txt
