"""Per-shape medians of the rocprofv3 --pmc passes of benchmarks/pmc_dgemm.sh (the d-wide GEMM family, dispatch i of
the GEMM kernels = shape i % 10 of dgemm_family.SHAPES) -> OUTDIR/gemm_dwide_pmc.json, which bench.py's `roofline`
entry reads (`traffic` = the launch-weighted mean HBM bytes per launch).

HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> B): on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane
streaming reads, WRITE_SIZE is exact for 16-B stores (MI355X_MICROARCH.md §HBM).
usage: python pmc_dgemm_json.py DIR COMMAND"""
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dgemm_family import SHAPES  # noqa: E402

d, cmd = sys.argv[1:3]
NS = len(SHAPES)


def per_shape(tag):
    rows = [r for r in csv.DictReader(open(os.path.join(d, f"dg_{tag}.csv"))) if "gemm" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    pos = {i: k % NS for k, i in enumerate(ids)}
    by = {}
    names = {}
    for r in rows:
        s = pos[int(r["Dispatch_Id"])]
        by.setdefault(s, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        names[s] = r["Kernel_Name"]
    return {s: {k: statistics.median(v) for k, v in c.items()} for s, c in by.items()}, names


data, names = {}, {}
for tag in ("fetch", "write", "sqa", "sqb"):
    got, nm = per_shape(tag)
    names.update(nm)
    for s, c in got.items():
        data.setdefault(s, {}).update(c)

M, dm, F = 32 * 373, 512, 2048
K_OF = [F, F, dm, dm, F, F, 3 * dm, dm, 2 * dm, dm]
OUT_B = [4, 4, 4, 4, 2, 2, 2, 2, 2, 2]       # fp32 residual-stream forwards (+ fp32 residual read), bf16 dgrads
shapes = {}
tot_hbm = tot_alg = 0.0
for s in range(NS):
    c = data.get(s, {})
    hbm = 2 * 1024 * c.get("FETCH_SIZE", 0) + 1024 * c.get("WRITE_SIZE", 0)
    K = K_OF[s]
    alg = 2.0 * (M * K + dm * K) + OUT_B[s] * M * dm * (2 if OUT_B[s] == 4 else 1)
    mf = c.get("SQ_INSTS_MFMA", 0) or 1
    shapes[SHAPES[s]] = {
        "K": K, "kernel": names.get(s, "?")[:120], "hbm_bytes": hbm, "algorithmic_bytes": alg,
        "counters": c,
        "valu_per_mfma": round(c.get("SQ_INSTS_VALU", 0) / mf, 2),
        "lds_per_mfma": round(c.get("SQ_INSTS_LDS", 0) / mf, 2),
        "bank_conflict_per_lds": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_INSTS_LDS", 1)), 3),
        "wait_any_frac": round(c.get("SQ_WAIT_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)), 3),
        "wait_inst_any_frac": round(c.get("SQ_WAIT_INST_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)), 3),
        "wait_inst_lds_frac": round(c.get("SQ_WAIT_INST_LDS", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)), 3),
        "tcc_hit_rate": round(c.get("TCC_HIT_sum", 0) / max(1, c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)), 3),
    }
    tot_hbm += hbm
    tot_alg += alg
rec = {
    "kernel": "d-wide GEMM family (" + ", ".join(sorted({v["kernel"][:60] for v in shapes.values()})) + ")",
    "shape_key": [M, dm, F, 17],
    "hbm_bytes_per_launch": tot_hbm / NS,
    "algorithmic_bytes_per_launch": tot_alg / NS,
    "shapes": shapes,
    "command": f"rocprofv3 --pmc <FETCH_SIZE | WRITE_SIZE | 9 SQ/GRBM | 6 SQ + 2 TCC> (four separate passes) -- {cmd}",
    "correction": "fetch_bytes = 2 * FETCH_SIZE * 1024 (gfx950 counts half of 16-B/lane streaming reads); "
                  "write_bytes = WRITE_SIZE * 1024",
}
with open(os.path.join(d, "gemm_dwide_pmc.json"), "w") as f:
    json.dump(rec, f, indent=1)
print("gemm_dwide_pmc.json", json.dumps({k: (v["hbm_bytes"], v["valu_per_mfma"], v["lds_per_mfma"],
                                             v["wait_any_frac"]) for k, v in shapes.items()}))
