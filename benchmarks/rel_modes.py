"""Rel-pos attention at the L60 shape (B 8, T 1498, H 8, dk 64, dropout 0.1): forward and backward under
cfm_attn_set_mode values (interleaved rounds, HIP-event medians).
    python benchmarks/rel_modes.py [--modes 0] [--reps 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402


def timeit(fn, n=10, warm=2):
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
    ap.add_argument("--modes", default="0")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--drop", type=float, default=0.1, help="attention dropout p (0: no hash in either pass)")
    a = ap.parse_args()
    modes = [int(m) for m in a.modes.split(",")]
    B, T, H, dk = 8, 1498, 8, 64
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to("cuda", torch.bfloat16)
    pos = (0.5 * torch.randn(2 * T - 1, H * dk, generator=g)).to("cuda", torch.bfloat16)
    pu = (0.3 * torch.randn(H * dk, generator=g)).cuda()
    pv = (0.3 * torch.randn(H * dk, generator=g)).cuda()
    do = torch.randn(B * T, H * dk, generator=g).to("cuda", torch.bfloat16)
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, pos, pu, pv, drop_p=a.drop, seed=3)
    res = {}
    for _ in range(a.reps):
        for m in modes:
            _lib.call("cfm_attn_set_mode", m)
            res.setdefault(f"fwd mode {m}", []).append(
                timeit(lambda: ops.attn_fwd(qkv, lens, B, T, H, dk, pos, pu, pv, drop_p=a.drop, seed=3)))
            res.setdefault(f"bwd mode {m}", []).append(
                timeit(lambda: ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, pos, pu, pv, drop_p=a.drop, seed=3)))
    _lib.call("cfm_attn_set_mode", 0)
    out = {}
    for k, v in res.items():
        t = sorted(v)[len(v) // 2]
        out[k] = round(t, 1)
        print(f"{k:16s} {t:8.1f} us")
    print("REL " + json.dumps(out))


if __name__ == "__main__":
    main()
