#!/bin/bash
# Same-box A/B of two libcfm builds (CFM_LIB) on the attention kernels alone: the L15 probe and the L60 rel-pos
# shape, interleaved.  usage: bash benchmarks/attn_lib_ab.sh BASE_SO [ROUNDS]
BASE=$1; R=${2:-2}
for r in $(seq 1 $R); do
  for lib in "$BASE" ""; do
    tag=${lib:-new}
    CFM_LIB=$lib timeout -k 10 300 python -u benchmarks/attn_probe.py 2>/dev/null | grep '^ATTN' | sed "s|^|[$tag] |" || exit 1
    CFM_LIB=$lib timeout -k 10 300 python -u benchmarks/rel_modes.py --modes 0 --reps 5 2>/dev/null | grep '^REL' | sed "s|^|[$tag] |" || exit 1
  done
done
