#!/bin/bash
# r03 PMC passes: attention kernels at the L15 shape (benchmarks/attn_rel_probe.py --l15 --none) and the
# bench roofline kernels (benchmarks/pmc_roofline.sh) -> gpurun_out/pmc_r03
set -o pipefail
O=$(pwd)/gpurun_out/pmc_r03; mkdir -p $O
timeout -k 10 600 bash benchmarks/pmc_kernels.sh $O/attn_l15 python3 $(pwd)/benchmarks/attn_rel_probe.py 3 --l15 --none > $O/attn_l15.txt 2>&1 || { echo "attn pmc failed"; tail $O/attn_l15.txt; exit 1; }
cat $O/attn_l15.txt
timeout -k 10 900 bash benchmarks/pmc_roofline.sh $O > $O/roofline.log 2>&1 || { echo "roofline pmc failed"; tail $O/roofline.log; exit 1; }
ls $O
