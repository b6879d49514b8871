#!/bin/bash
# same-box A/B of the round-5 closing tree (git worktree at ab/r05tree, its own libcfm.so) against this tree, every
# benchmarked configuration, interleaved
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$(realpath -m "${1:-gpurun_out/ab_rounds}"); mkdir -p $O
ms() { python -c "import json; r=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1'.split('/')[-1], r['ms_per_step'], r['valid'])"; }
one() {   # tag tree args...
  local tag=$1 tree=$2; shift 2
  (cd $tree && timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err) && ms $O/$tag.json || { tail -5 $O/$tag.err; exit 1; }
}
for rep in 1 2; do
  for t in r05 r06; do
    tree=$R; [ $t = r05 ] && tree=$R/ab/r05tree
    one L15_$t.$rep $tree --steps 20 --warmup 5
    one S15_$t.$rep $tree --config S15 --steps 20 --warmup 5
    one M15sa_$t.$rep $tree --config M15 --specaug --steps 20 --warmup 5
  done
done
for t in r05 r06; do
  tree=$R; [ $t = r05 ] && tree=$R/ab/r05tree
  one L60_$t $tree --config L60 --steps 10 --warmup 3
  one L60fp8_$t $tree --config L60 --fp8 --steps 10 --warmup 3
done
