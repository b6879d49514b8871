#!/bin/bash
# L60 bench.py with the dpos kernel summing utterance groups per workgroup (default) vs one utterance per
# workgroup (cfm_attn_set_mode bit 9 = 512), one box, alternating
set -e
for m in 0 512 0 512; do
  timeout -k 10 400 python bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline --attn-mode $m > /tmp/dg.json
  grep '^{' /tmp/dg.json | python3 -c "
import json,sys; r=json.load(sys.stdin); print('attn_mode', $m, 'ms/step', r['ms_per_step'])"
done
