"""Where do torch fill kernels come from?  Runs bench.py eagerly (1 warm-up + 2 steps) under the torch
profiler and prints the Python stacks of aten::fill_ / zero_ calls, most frequent first."""
import collections
import runpy
import sys

from torch.profiler import ProfilerActivity, profile

sys.argv = ["bench.py", "--eager", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    runpy.run_path("bench.py", run_name="__main__")
cnt = collections.Counter()
for e in prof.events():
    if e.name in ("aten::fill_", "aten::zero_"):
        st = [s for s in (e.stack or []) if "torch/" not in s][:4] or list(e.stack or [])[:4]
        if not st:
            par = e.cpu_parent
            chain = []
            while par is not None and len(chain) < 5:
                chain.append(par.name)
                par = par.cpu_parent
            st = chain
        cnt[(e.name, " <- ".join(st))] += 1
for (n, st), c in cnt.most_common(15):
    print(c, n, st)

# stackless fills (autograd worker thread): the ops issued just before them on the same thread
evs = sorted([e for e in prof.events()], key=lambda e: (e.thread, e.time_range.start))
ctx = collections.Counter()
for i, e in enumerate(evs):
    if e.name in ("aten::fill_", "aten::zero_") and not e.stack and e.cpu_parent is None:
        prev = [evs[j].name for j in range(max(0, i - 4), i) if evs[j].thread == e.thread]
        ctx[(e.name, " | ".join(prev))] += 1
print("--- stackless fills by preceding ops")
for (n, p), c in ctx.most_common(12):
    print(c, n, "after:", p)
