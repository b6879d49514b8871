"""Grouped weight-gradient launch lab: the L15 backward's 17 layers x 8 GEMMs (M = 11,936 tokens) with DISTINCT
operands per layer (as in the step: 6.4 GB of dY / X, beyond the 256 MiB Infinity Cache), timed with HIP events
over back-to-back launches; layer counts 14 / 16 / 17 show whether the launch time follows the tile count or the
number of 256-CU rounds (1,288 / 1,472 / 1,564 tiles = 5.03 / 5.75 / 6.11 rounds).
    python benchmarks/wgrad_lab.py [--modes 3] [--layers 14,16,17] [--reps 5]
A mode with bit 30 set runs the UNPLANNED launch (ops.WGRAD_PLAN = False: tiles in task order, XCD-contiguous ids);
the rest of the value goes to cfm_gemm_set_mode."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="3")
    ap.add_argument("--layers", default="14,16,17")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", action="store_true", help="compare every mode's dW / db with mode 3's")
    a = ap.parse_args()
    modes = [int(m) for m in a.modes.split(",")]
    M, d, F = 32 * 373, 512, 2048
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [(F, d), (d, F)] * 2 + [(3 * d, d), (d, d), (2 * d, d), (d, d)]   # dW (N, K) per layer
    Lmax = max(int(x) for x in a.layers.split(","))
    pairs = [(torch.randn(M, n, device="cuda", generator=g).to(torch.bfloat16),
              torch.randn(M, k, device="cuda", generator=g).to(torch.bfloat16)) for _ in range(Lmax) for n, k in shapes]
    out = {}
    for nl in (int(x) for x in a.layers.split(",")):
        pp = pairs[: 8 * nl]
        fl = sum(2.0 * M * dy.shape[1] * x.shape[1] for dy, x in pp)
        tiles = sum(_lib.load().cfm_wgrad_group_tiles(dy.shape[1], x.shape[1]) for dy, x in pp)
        res = {m: [] for m in modes}
        grps = {m: ops.WgradGroup() for m in modes}
        ref = None
        for rep in range(a.reps):
            for m in modes:
                _lib.call("cfm_gemm_set_mode", m & ~(1 << 30))
                ops.WGRAD_PLAN = not (m >> 30) & 1
                grp = grps[m]

                def run():
                    outs = [grp.add(dy, x) for dy, x in pp]
                    grp.flush()
                    return outs
                for _ in range(2):
                    o = run()
                torch.cuda.synchronize()
                if a.check and rep == 0:
                    if ref is None:
                        ref = [(w.clone(), b.clone()) for w, b in o]
                    else:
                        err = max(max((w - rw).abs().max().item(), (b - rb).abs().max().item())
                                  for (w, b), (rw, rb) in zip(o, ref))
                        print(f"layers {nl} mode {m}: max |diff| vs first mode {err:.3e}", flush=True)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    run()
                e.record()
                torch.cuda.synchronize()
                res[m].append(s.elapsed_time(e) / 5)
        for m in modes:
            t = sorted(res[m])[len(res[m]) // 2]
            out[f"L{nl}_m{m}"] = round(t, 4)
            print(f"layers {nl:2d} ({tiles} tiles = {tiles / 256:.2f} rounds) mode {m:9d}: {t:7.3f} ms  "
                  f"{fl / t / 1e9:6.0f} TF/s  {fl / t / 1e9 / 2500:.3f} of peak", flush=True)
    _lib.call("cfm_gemm_set_mode", 3)
    print("WGRADLAB " + json.dumps(out))


if __name__ == "__main__":
    main()
