#!/bin/bash
# L60 bench.py with the batched rel-pos tables / grouped dW_pos (default) vs the per-layer GEMMs
# (CFM_REL_BATCH=0), one box, alternating
set -e
for v in 1 0 1 0; do
  CFM_REL_BATCH=$v timeout -k 10 400 python bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline > /tmp/rb.json
  grep '^{' /tmp/rb.json | python3 -c "
import json,sys; r=json.load(sys.stdin); print('REL_BATCH', $v, 'ms/step', r['ms_per_step'], 'ctc', r['ctc_head']['ms'], 'wgrad', r['roofline_wgrad']['avg_launch_ms_live'])"
done
