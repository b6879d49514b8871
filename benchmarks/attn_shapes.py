"""Attention timing at the step's shapes: libcfm fwd / bwd (dropout 0.1 and 0) and, for scale, torch SDPA
(the ROCm flash backend) on the same (B, H, T, dk).  Also the libcfm forward's staging-only and no-store
timing modes (cfm_attn_set_mode bits 1, 2).   python benchmarks/attn_shapes.py [--T 373 --B 32]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

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
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=373)
    ap.add_argument("--H", type=int, default=8)
    ap.add_argument("--dk", type=int, default=64)
    a = ap.parse_args()
    B, T, H, dk = a.B, a.T, a.H, a.dk
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * T, 3 * H * dk, device="cuda", generator=g).to(torch.bfloat16)
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    fl = 4.0 * B * H * T * T * dk
    out = {}
    for p in (0.1, 0.0):
        o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=p, seed=3)
        do = torch.randn_like(o)
        tf = timeit(lambda: ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=p, seed=3))
        tb = timeit(lambda: ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=p, seed=3))
        out[f"fwd_p{p}"], out[f"bwd_p{p}"] = round(tf, 2), round(tb, 2)
        print(f"libcfm p={p}: fwd {tf:7.1f} us {fl / tf / 1e6:6.0f} TF/s | bwd {tb:7.1f} us {2.5 * fl / tb / 1e6:6.0f} TF/s")
    for mode, tag in ((32, "LDS-DMA staged (A/B)"), (2, "staging only"), (4, "no epilogue stores")):
        _lib.call("cfm_attn_set_mode", mode)
        t = timeit(lambda: ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=3))
        out[f"fwd_mode{mode}"] = round(t, 2)
        print(f"libcfm fwd {tag}: {t:7.1f} us")
    _lib.call("cfm_attn_set_mode", 0)
    q, k, v = (qkv.view(B, T, 3, H, dk)[:, :, i].transpose(1, 2).contiguous().requires_grad_() for i in range(3))
    try:
        ts = timeit(lambda: F.scaled_dot_product_attention(q, k, v))
        y = F.scaled_dot_product_attention(q, k, v)
        gy = torch.randn_like(y)
        tsb = timeit(lambda: torch.autograd.grad(y, (q, k, v), gy, retain_graph=True))
        out["sdpa_fwd"], out["sdpa_bwd"] = round(ts, 2), round(tsb, 2)
        print(f"torch SDPA (no dropout): fwd {ts:7.1f} us {fl / ts / 1e6:6.0f} TF/s | bwd {tsb:7.1f} us")
    except Exception as e:   # noqa: BLE001
        print("torch SDPA unavailable:", repr(e)[:200])
    print(json.dumps({"B": B, "T": T, "H": H, "dk": dk, "us": out}))


if __name__ == "__main__":
    main()
