#!/bin/bash
# same-box A/B of the bf16 residual stream (CFM_RES_BF16) on L15 and L60, interleaved
set -o pipefail
O=${1:-gpurun_out/ab_res}; mkdir -p $O
ms() { python -c "import json; r=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1', r['ms_per_step'], r['valid'])"; }
for rep in 1 2; do
  for v in 0 1; do
    CFM_RES_BF16=$v timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/l15_res$v.$rep.json && ms $O/l15_res$v.$rep.json || exit 1
  done
done
for v in 0 1; do
  CFM_RES_BF16=$v timeout -k 10 200 python -u bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline > $O/l60_res$v.json && ms $O/l60_res$v.json || exit 1
done
