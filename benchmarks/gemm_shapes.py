"""Per-shape timing of the encoder step's GEMM kinds at Conformer-L / 15 s (M = 11,936 tokens), as the step
issues them (epilogues included).  HIP events over N launches, median of R repetitions.  Pick the library with
CFM_LIB=... for same-box A/B of builds (benchmarks/ab_gemm.sh).
    python benchmarks/gemm_shapes.py [--reps 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402
from nn_conformer_for_speech_recognition_amd._lib import ACT_SILU  # noqa: E402


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
    return s.elapsed_time(e) / n * 1e3        # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--torch", action="store_true", help="also time torch (hipBLASLt) on the bare GEMMs")
    ap.add_argument("--mode", type=int, default=None, help="cfm_gemm_set_mode value")
    a = ap.parse_args()
    if a.mode is not None:
        from nn_conformer_for_speech_recognition_amd import _lib
        _lib.call("cfm_gemm_set_mode", a.mode)
    M, d, F = 32 * 373, 512, 2048
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)

    def rn(*s, dt=bf, sc=1.0):
        return (torch.randn(*s, device="cuda", generator=g) * sc).to(dt)
    x512, x2048 = rn(M, d), rn(M, F)
    w_up, w_dn = rn(F, d, sc=0.05), rn(d, F, sc=0.05)
    w_up_t, w_dn_t = w_up.t().contiguous(), w_dn.t().contiguous()
    w_qkv, w_o = rn(3 * d, d, sc=0.05), rn(d, d, sc=0.05)
    b_up, b_dn, b_qkv = rn(F, dt=torch.float32), rn(d, dt=torch.float32), rn(3 * d, dt=torch.float32)
    res = rn(M, d, dt=torch.float32)
    y_up, pre = torch.empty(M, F, device="cuda", dtype=bf), torch.empty(M, F, device="cuda", dtype=bf)
    y_dn = torch.empty(M, d, device="cuda", dtype=torch.float32)
    qkv = torch.empty(M, 3 * d, device="cuda", dtype=bf)
    g2 = rn(M, d)
    da = torch.empty(M, F, device="cuda", dtype=bf)
    dxn = torch.empty(M, d, device="cuda", dtype=bf)
    cases = {
        "ffn_up fwd (bias+silu+drop+pre)": (2 * M * F * d, lambda: ops.linear(x512, w_up, b_up, act=ACT_SILU, pre=pre,
                                                                            drop_p=0.1, seed=1, out=y_up)),
        "ffn_down fwd (fp32 out, drop, 0.5, residual)": (2 * M * F * d, lambda: ops.linear(
            x2048, w_dn, b_dn, out=y_dn, drop_p=0.1, seed=2, out_scale=0.5, residual=res)),
        "qkv fwd": (2 * M * 3 * d * d, lambda: ops.linear(x512, w_qkv, b_qkv, out=qkv)),
        "out fwd (fp32, residual)": (2 * M * d * d, lambda: ops.linear(x512, w_o, b_dn, out=y_dn, residual=res)),
        "ffn_down dgrad (silu' + drop epilogue)": (2 * M * F * d, lambda: ops.linear_dgrad(
            g2, w_dn, pre=pre, act_grad=True, drop_p=0.1, seed=1, wt=w_dn_t, out=da)),
        "ffn_up dgrad": (2 * M * F * d, lambda: ops.linear_dgrad(da, w_up, wt=w_up_t, out=dxn)),
    }
    res_t = {k: [] for k in cases}
    for _ in range(a.reps):
        for k, (fl, fn) in cases.items():
            res_t[k].append(timeit(fn))
    out = {}
    for k, (fl, fn) in cases.items():
        t = sorted(res_t[k])[len(res_t[k]) // 2]
        out[k] = round(t, 2)
        print(f"{k:48s} {t:8.2f} us {fl / t / 1e6:7.0f} TF/s")
    if a.torch:
        import torch.nn.functional as tF
        tc = {"torch ffn_up fwd (bias only)": (2 * M * F * d, lambda: tF.linear(x512, w_up)),
              "torch ffn_down fwd (bf16 out)": (2 * M * F * d, lambda: tF.linear(x2048, w_dn)),
              "torch qkv fwd": (2 * M * 3 * d * d, lambda: tF.linear(x512, w_qkv)),
              "torch out fwd": (2 * M * d * d, lambda: tF.linear(x512, w_o)),
              "torch ffn_down dgrad (da = g2 W2)": (2 * M * F * d, lambda: torch.mm(g2, w_dn)),
              "torch ffn_up dgrad (dx = da W1)": (2 * M * F * d, lambda: torch.mm(da, w_up)),
              "torch wgrad ffn_up (dW1 = da^T x)": (2 * M * F * d, lambda: torch.mm(da.t(), x512)),
              "torch wgrad ffn_down (dW2 = g2^T h)": (2 * M * F * d, lambda: torch.mm(g2.t(), x2048))}
        for k, (fl, fn) in tc.items():
            t = sorted(timeit(fn) for _ in range(a.reps))[a.reps // 2]
            out[k] = round(t, 2)
            print(f"{k:48s} {t:8.2f} us {fl / t / 1e6:7.0f} TF/s")
    # grouped weight gradients of one layer (8 GEMMs) as the step launches them
    grp = ops.WgradGroup()
    pairs = [(g2, x2048), (da, x512), (g2, x2048), (da, x512), (qkv, x512), (g2, x512), (rn(M, 2 * d), x512),
             (g2, x512)]
    fl = sum(2 * M * dy.shape[1] * x.shape[1] for dy, x in pairs)

    def wg():
        for dy, x in pairs:
            grp.add(dy, x)
        grp.flush()
    t = sorted(timeit(wg, n=10) for _ in range(a.reps))[a.reps // 2]
    out["wgrad group (1 layer, 8 GEMMs)"] = round(t, 2)
    print(f"{'wgrad group (1 layer, 8 GEMMs)':48s} {t:8.2f} us {fl / t / 1e6:7.0f} TF/s")
    print(json.dumps({"lib": os.environ.get("CFM_LIB", "default"), "mode": a.mode, "us": out}))


if __name__ == "__main__":
    main()
