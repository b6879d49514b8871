#!/bin/bash
# Same-box A/B of two libcfm builds on the GEMM shapes (interleaved rounds).
# usage: bash benchmarks/ab_gemm.sh ROUNDS LIB_A LIB_B
R=$1; A=$2; B=$3
for r in $(seq 1 $R); do
  for L in $A $B; do
    CFM_LIB=$L timeout -k 10 120 python benchmarks/gemm_shapes.py --reps 3 | tail -1 || exit 1
  done
done
