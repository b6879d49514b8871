"""Per-dispatch medians of the rocprofv3 --pmc passes written by benchmarks/pmc_roofline.sh, for the
dispatches whose kernel name contains a filter string -> one JSON record that bench.py's roofline
entries read (matched on shape_key and the kernel name recorded here).

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> B): on gfx950 FETCH_SIZE counts half the bytes
of 16-B-per-lane streaming reads, WRITE_SIZE is exact for 16-B stores (MI355X_MICROARCH.md §HBM).
usage: python pmc_to_json.py DIR PREFIX KERNEL_FILTER OUT_NAME COMMAND [ALGORITHMIC_BYTES_PER_LAUNCH]
env PMC_AGG=mean: per-dispatch MEANS instead of medians (a family of several shapes, whose algorithmic bytes are a
mean per launch); env PMC_SHAPE="M,d,ffn,L": the bench config's shape key (default L15's)."""
import csv
import json
import os
import statistics
import sys

d, pre, filt, out_name, cmd = sys.argv[1:6]
alg = float(sys.argv[6]) if len(sys.argv) > 6 else None


def medians(tag):
    rows = [r for r in csv.DictReader(open(os.path.join(d, f"{pre}_{tag}.csv"))) if filt in r["Kernel_Name"]]
    by = {}
    for r in rows:
        by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    agg = statistics.mean if os.environ.get("PMC_AGG") == "mean" else statistics.median
    return {k: agg(v) for k, v in by.items()}, (rows[0]["Kernel_Name"] if rows else "?"), \
        len({r.get("Dispatch_Id", i) for i, r in enumerate(rows)})


fetch, kname, nf = medians("fetch")
write, _, nw = medians("write")
mfma, _, nm = medians("mfma")
rec = {
    "kernel": kname,
    "shape_key": [int(v) for v in os.environ["PMC_SHAPE"].split(",")] if os.environ.get("PMC_SHAPE") else
                 [32 * 373, 512, 2048, 17],       # M tokens, d, ffn, layers (bench.py L15)
    "aggregate": os.environ.get("PMC_AGG", "median"),
    "FETCH_SIZE_KiB_median": fetch.get("FETCH_SIZE"), "WRITE_SIZE_KiB_median": write.get("WRITE_SIZE"),
    "dispatches": {"fetch": nf, "write": nw, "mfma": nm},
    "SQ_INSTS_MFMA_median": mfma.get("SQ_INSTS_MFMA"),
    "SQ_VALU_MFMA_BUSY_CYCLES_median": mfma.get("SQ_VALU_MFMA_BUSY_CYCLES"),
    "SQ_BUSY_CYCLES_median": mfma.get("SQ_BUSY_CYCLES"),
    "GRBM_GUI_ACTIVE_median": mfma.get("GRBM_GUI_ACTIVE"),
    "hbm_bytes_per_launch": 2 * 1024 * fetch.get("FETCH_SIZE", 0) + 1024 * write.get("WRITE_SIZE", 0),
    "command": f"rocprofv3 --pmc <FETCH_SIZE | WRITE_SIZE | SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES "
               f"GRBM_GUI_ACTIVE> (three separate passes) -- {cmd}",
    "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": None if not alg else round(
        (2 * 1024 * fetch.get("FETCH_SIZE", 0) + 1024 * write.get("WRITE_SIZE", 0)) / alg, 3),
    "correction": "fetch_bytes = 2 * FETCH_SIZE * 1024 (gfx950 counts half of 16-B/lane streaming reads); "
                  "write_bytes = WRITE_SIZE * 1024",
}
with open(os.path.join(d, out_name), "w") as f:
    json.dump(rec, f, indent=1)
print(out_name, json.dumps(rec)[:400])
