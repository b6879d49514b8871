"""The encoder's wide-output, short-reduction GEMMs at L15 (M = 11,936 tokens, K = 512) as the step issues them:
FFN-up forward (N 2048: bias + SiLU + pre-activation + dropout, two bf16 outputs), FFN-down data gradient (N 2048:
silu'(pre) + dropout), QKV forward (N 1536, bias) and pointwise-conv-1 forward (N 1024, bias), timed under several
cfm_gemm_set_mode values in one process (interleaved rounds).

    python benchmarks/wide_gemm.py [--modes 3,11,83] [--reps 5] [--variants]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402


def timeit(fn, n=20, warm=3):
    """Device time per call: n calls captured in one HIP graph and replayed (the Python / ctypes launch path costs
    ~12 us per call, more than the short-K GEMMs themselves: event timing of eager launches floors there)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3        # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="3,11")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", action="store_true")
    a = ap.parse_args()
    modes = [int(m) for m in a.modes.split(",")]
    M, d, F = 32 * 373, 512, 2048
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)

    def rn(*s, dt=bf, sc=1.0):
        return (torch.randn(*s, device="cuda", generator=g) * sc).to(dt)
    x = rn(M, d)
    w_up, w_qkv, w_pw1 = rn(F, d, sc=0.05), rn(3 * d, d, sc=0.05), rn(2 * d, d, sc=0.05)
    w_dn_t = rn(F, d, sc=0.05)                  # (K = d ... ) K-major copy of W2^T: (F, d)
    b_up, b_qkv, b_pw1 = rn(F, dt=torch.float32), rn(3 * d, dt=torch.float32), rn(2 * d, dt=torch.float32)
    y, pre = torch.empty(M, F, device="cuda", dtype=bf), torch.empty(M, F, device="cuda", dtype=bf)
    g2 = rn(M, d)
    da = torch.empty(M, F, device="cuda", dtype=bf)
    qkv = torch.empty(M, 3 * d, device="cuda", dtype=bf)
    a1 = torch.empty(M, 2 * d, device="cuda", dtype=bf)
    ops.linear(x, w_up, b_up, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=1, out=y)
    cases = {
        "ffn_up_fwd": (2 * M * F * d, lambda: ops.linear(x, w_up, b_up, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=1,
                                                          out=y)),
        "ffn_down_dgrad": (2 * M * F * d, lambda: ops.gemm(g2, w_dn_t, da, M, F, d, pre=pre, act_grad=True, drop_p=0.1,
                                                           seed=1)),
        "qkv_fwd": (2 * M * 3 * d * d, lambda: ops.linear(x, w_qkv, b_qkv, out=qkv)),
        "pw1_fwd": (2 * M * 2 * d * d, lambda: ops.linear(x, w_pw1, b_pw1, out=a1)),
    }
    if a.variants:   # the FFN-up epilogue taken apart: bias only, + SiLU, + pre-activation store, + dropout
        cases.update({
            "up_bias": (2 * M * F * d, lambda: ops.linear(x, w_up, b_up, out=y)),
            "up_silu": (2 * M * F * d, lambda: ops.linear(x, w_up, b_up, act=ops.ACT_SILU, out=y)),
            "up_silu_pre": (2 * M * F * d, lambda: ops.linear(x, w_up, b_up, act=ops.ACT_SILU, pre=pre, out=y)),
            "up_silu_drop": (2 * M * F * d, lambda: ops.linear(x, w_up, b_up, act=ops.ACT_SILU, drop_p=0.1, seed=1,
                                                                out=y)),
        })
    res = {m: {k: [] for k in cases} for m in modes}
    for _ in range(a.reps):
        for m in modes:
            _lib.call("cfm_gemm_set_mode", m)
            for k, (fl, fn) in cases.items():
                res[m][k].append(timeit(fn))
    _lib.call("cfm_gemm_set_mode", 3)
    out = {}
    for m in modes:
        row = {}
        for k, (fl, _) in cases.items():
            t = sorted(res[m][k])[len(res[m][k]) // 2]
            row[k] = round(t, 2)
        out[m] = row
        print(f"mode {m:8d}: " + "  ".join(f"{k} {v:7.2f} us" for k, v in row.items()))
    print("WIDE " + json.dumps(out))


if __name__ == "__main__":
    main()
