"""Attention timing experiments at L15 (B 32, T 373, 8 heads, dk 64, dropout 0.1): the forward under the
cfm_attn_set_mode dbg bits (0 full, 2 staging only, 4 no epilogue stores) and the backward (dQ + dK/dV), HIP-event
medians of interleaved rounds.
    python benchmarks/attn_probe.py [--reps 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402


def timeit(fn, n=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--T", type=int, default=373)
    ap.add_argument("--B", type=int, default=32)
    a = ap.parse_args()
    B, T, H, dk = a.B, a.T, 8, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * T, 3 * H * dk, device="cuda", generator=g).to(torch.bfloat16)
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=3)
    do = torch.randn(B * T, H * dk, device="cuda", generator=g).to(torch.bfloat16)
    cases = {}
    for mode, tag in ((0, "fwd"), (2, "fwd staging only"), (4, "fwd no stores")):
        cases[tag] = (mode, lambda: ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=3))
    cases["bwd (D + dQ + dK/dV)"] = (0, lambda: ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=0.1, seed=3))
    cases["fwd p=0"] = (0, lambda: ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.0, seed=3))
    cases["bwd p=0"] = (0, lambda: ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=0.0, seed=3))
    res = {k: [] for k in cases}
    for _ in range(a.reps):
        for k, (mode, fn) in cases.items():
            _lib.call("cfm_attn_set_mode", mode)
            res[k].append(timeit(fn))
    _lib.call("cfm_attn_set_mode", 0)
    fl = 4.0 * B * H * T * T * dk
    out = {}
    for k in cases:
        t = sorted(res[k])[len(res[k]) // 2]
        out[k] = round(t, 2)
        mult = 2.5 if k.startswith("bwd") else 1.0
        print(f"{k:24s} {t:8.2f} us  {mult * fl / t / 1e6:6.0f} TF/s")
    print("ATTN " + json.dumps(out))


if __name__ == "__main__":
    main()
