"""Summarise a rocprofv3 --kernel-trace CSV of a bench.py run into the per-family figures bench.py's roofline entries
quote beside their live probes (`avg_launch_ms_trace`).

    python profiles/summarize_trace.py KERNEL_TRACE.csv OUT.json --config L15 --warmup W --steps K

The bench run dispatches, in order: W eager warm-up steps, one graph replay, K timed replays, then K replays of the
probe graph, where every probed launch sits between two probe_slot_kernel dispatches.  The probe brackets name each
family's kernel signatures (kernel name + workgroup count; a launch may be several dispatches); a step ends at the grouped weight-gradient launch (one
per step).  Family figures are the mean durations (End - Start, the kernel trace's own clock) of those signatures'
UNBRACKETED dispatches in the K timed replays, i.e. in the timed graph that carries no probe kernels:
* wgrad  -- the grouped weight-gradient launch (gemm_pipe_kernel<256, 32, 4, 1, ...> + its split-slab reduction);
* ffn_up -- the FFN up-projection forward (gemm_pipe_kernel<256, 32, 3, 2, ...>, the bracketed signature only);
* fp8    -- the fp8 (MX e4m3) forward GEMMs of a --fp8 run (gemm_pipe_kernel<..., F8 = true, ...>);
* dwide  -- every other bracketed signature (the d-wide GEMM family of bench.py's `roofline`).
Also written: every signature's launches per timed step and mean duration, and the timed steps' kernel time."""
import argparse
import csv
import hashlib
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("out")
ap.add_argument("--config", required=True)
ap.add_argument("--warmup", type=int, required=True)
ap.add_argument("--steps", type=int, required=True)
ap.add_argument("--lib", default=None, help="libcfm.so the traced run loaded: its md5 binds the summary to that build")
a = ap.parse_args()

WGRAD, FFNUP, PROBE = "gemm_pipe_kernel<256, 32, 4, 1,", "gemm_pipe_kernel<256, 32, 3, 2,", "probe_slot_kernel"


def wgs(r):
    n = 1
    for ax in "XYZ":
        n *= max(1, int(r[f"Grid_Size_{ax}"]) // max(1, int(r[f"Workgroup_Size_{ax}"])))
    return n


rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
disp = []
step = 0
for r in rows:
    name = r["Kernel_Name"]
    disp.append({"name": name, "sig": (name, wgs(r)), "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                 "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]), "step": step})
    if WGRAD in name:
        step += 1
# bracketed: the probed launch of a (stamp, launch..., accumulate) group -- parsed left to right: an opening probe
# kernel, every non-probe dispatch up to the next probe kernel (the grouped weight-gradient launch is two: the GEMM
# and its split-slab reduction), the closing probe kernel; an unprobed dispatch between two groups is skipped and
# the calibration pairs (two probe kernels back to back) hold nothing
for d in disp:
    d["bracketed"] = False
groups = []
i = 0
while i < len(disp):
    if PROBE not in disp[i]["name"]:
        i += 1
        continue
    j = i + 1
    while j < len(disp) and PROBE not in disp[j]["name"]:
        j += 1
    if j >= len(disp):
        break
    if j > i + 1:
        for d in disp[i + 1:j]:
            d["bracketed"] = True
        groups.append(tuple(d["sig"] for d in disp[i + 1:j]))
    i = j + 1
def is_f8(name):
    """gemm_pipe_kernel's 11th template argument is F8 (fp8 e4m3 operands, the --fp8 forward GEMMs)."""
    if "gemm_pipe_kernel<" not in name:
        return False
    args = name.split("gemm_pipe_kernel<", 1)[1].split(">", 1)[0].split(", ")
    return len(args) > 10 and args[10] == "true"


fam_groups = {"wgrad": set(), "ffn_up": set(), "dwide": set(), "fp8": set()}
for g in groups:
    n = g[0][0]
    fam_groups["wgrad" if WGRAD in n else "fp8" if is_f8(n) else "ffn_up" if FFNUP in n else "dwide"].add(g)
t0, t1 = a.warmup + 1, a.warmup + 1 + a.steps          # timed replays: steps [t0, t1)
timed = [d for d in disp if t0 <= d["step"] < t1 and not d["bracketed"] and PROBE not in d["name"]]
if not timed:
    raise SystemExit("no timed steps found (check --warmup / --steps)")
K = a.steps
fams = {}
for f, gs in fam_groups.items():
    members = {sg for g in gs for sg in g}
    heads = {g[0] for g in gs}
    ns = [d["ns"] for d in timed if d["sig"] in members]
    launches = [d["ns"] for d in timed if d["sig"] in heads]
    if launches:
        fams[f] = {"avg_ns": sum(ns) / len(launches), "launches_per_step": len(launches) / K,
                   "ms_per_step": sum(ns) / K / 1e6,
                   "signatures": sorted(f"{s[0][:110]} [{s[1]} WGs]" for s in members)}
by = {}
for d in timed:
    by.setdefault(d["sig"], []).append(d["ns"])
sigs = sorted(by.items(), key=lambda kv: -sum(kv[1]))
span = (max(d["end"] for d in timed) - min(d["start"] for d in timed)) / K / 1e6
lib_md5 = hashlib.md5(open(a.lib, "rb").read()).hexdigest() if a.lib else None
rec = {"config": a.config, "source": a.trace, "lib_md5": lib_md5, "timed_steps": K, "warmup": a.warmup,
       "kernel_ms_per_step": sum(d["ns"] for d in timed) / K / 1e6,
       "first_start_to_last_end_ms_per_step": span,
       "families": fams,
       "kernels": [{"name": s[0][:160], "workgroups": s[1], "launches_per_step": len(v) / K,
                    "avg_us": sum(v) / len(v) / 1e3, "ms_per_step": sum(v) / K / 1e6} for s, v in sigs]}
with open(a.out, "w") as f:
    json.dump(rec, f, indent=1)
print(f"{a.config}: kernel time {rec['kernel_ms_per_step']:.3f} ms/step, span {span:.3f} ms/step over {K} timed steps")
for f, v in fams.items():
    print(f"  {f:7s} {v['launches_per_step']:6.1f}/step  avg {v['avg_ns'] / 1e3:8.2f} us  {v['ms_per_step']:.3f} ms/step")
for k in rec["kernels"][:40]:
    print(f"  {k['ms_per_step']:8.3f} ms/step  {k['launches_per_step']:6.1f}/step  avg {k['avg_us']:8.1f} us  "
          f"[{k['workgroups']}] {k['name'][:100]}")
