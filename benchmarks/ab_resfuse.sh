#!/bin/bash
# same-box A/B of the residual add moved into the next LayerNorm (CFM_RES_FUSE, conformer.py) on L15, S15, M15 and L60,
# interleaved; then the residual-epilogue probe
set -o pipefail
O=${1:-gpurun_out/ab_resfuse}; mkdir -p $O
ms() { python -c "import json; r=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1', r['ms_per_step'], r['valid'])"; }
for rep in 1 2; do
  for v in 0 1; do
    CFM_RES_FUSE=$v timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/l15_f$v.$rep.json && ms $O/l15_f$v.$rep.json || exit 1
  done
done
for c in S15 M15; do
  for v in 0 1; do
    CFM_RES_FUSE=$v timeout -k 10 150 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${c}_f$v.json && ms $O/${c}_f$v.json || exit 1
  done
done
for v in 0 1; do
  CFM_RES_FUSE=$v timeout -k 10 200 python -u bench.py --config L60 --steps 10 --warmup 3 --no-cpu-baseline > $O/l60_f$v.json && ms $O/l60_f$v.json || exit 1
done
timeout -k 10 120 python -u benchmarks/res_epi_probe.py > $O/res_epi_probe.txt 2>&1 && cat $O/res_epi_probe.txt
