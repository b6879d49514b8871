#!/bin/bash
set -e
R=$(pwd)
for cfg in L15 L60; do
  for lib in new old; do
    if [ $lib = old ]; then export CFM_LIB=$R/benchmarks/libcfm_ab.so; else unset CFM_LIB; fi
    timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > /tmp/ctcab.json
    grep '^{' /tmp/ctcab.json | python3 -c "
import json,sys; r=json.load(sys.stdin); print('$cfg', '$lib', 'ms/step', r['ms_per_step'], 'ctc_head ms', r['ctc_head']['ms'])"
  done
done
