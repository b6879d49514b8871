#!/bin/bash
# Same-box A/B of a base libcfm build (CFM_LIB=BASE_SO) against the in-tree build: L15 (and optional extra config)
# bench lines interleaved, then a rocprofv3 kernel-stats pass of each build.
# usage: bash benchmarks/ab_lib_l15.sh BASE_SO OUTDIR [ROUNDS] [extra bench args]
set -o pipefail
BASE=$(realpath "$1"); O=$(realpath -m "$2"); R=${3:-2}; shift 3; EXTRA="$*"
mkdir -p "$O"; cd "$(dirname "$0")/.."
for r in $(seq 1 $R); do
  for lib in "$BASE" ""; do
    tag=$([ -n "$lib" ] && echo base || echo new)
    CFM_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $EXTRA > "$O/bench_$tag.$r.json" 2> "$O/bench_$tag.$r.err" || { echo "bench failed $tag"; exit 1; }
    echo "[$tag] $(python3 -c "import json; r=json.loads([l for l in open('$O/bench_$tag.$r.json') if l.startswith('{')][-1]); print(r['ms_per_step'], r['valid'])")"
  done
done
for lib in "$BASE" ""; do
  tag=$([ -n "$lib" ] && echo base || echo new)
  D=/tmp/abprof_$tag_$$
  (cd /tmp && export TMPDIR=/tmp && CFM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $OLDPWD/bench.py --steps 10 --warmup 3 --no-cpu-baseline $EXTRA > $O/prof_$tag.log 2>&1) || { echo "prof failed $tag"; exit 1; }
  cp "$(find $D -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats_$tag.csv"
  rm -rf $D
done
python3 - "$O" <<'PY'
import csv, sys
o = sys.argv[1]
def load(tag):
    d = {}
    for r in csv.DictReader(open(f"{o}/kernel_stats_{tag}.csv")):
        d[r["Name"][:120]] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6)
    return d
b, n = load("base"), load("new")
rows = sorted(set(b) | set(n), key=lambda k: -(n.get(k, b.get(k))[2]))
print(f"{'base us':>9} {'new us':>9} {'calls':>6}  kernel")
for k in rows[:30]:
    bb, nn = b.get(k), n.get(k)
    print(f"{(bb[0] if bb else float('nan')):9.2f} {(nn[0] if nn else float('nan')):9.2f} {(nn or bb)[1]:6d}  {k[:100]}")
PY
