"""The d-wide-output GEMM family of one Conformer-L layer at L15 (M = 11,936 tokens, N = d = 512), exactly as the
step issues it (epilogues included): FFN-down forward x2 (K 2048, bias + dropout + 0.5 + fp32 residual),
out-projection and pointwise-conv-2 forward (K 512, bias (+ dropout) + fp32 residual), and the data gradients of
FFN-up x2 (K 2048), QKV (K 1536), out-projection (K 512), pointwise-conv-1 (K 1024), pointwise-conv-2 (K 512).

    python benchmarks/dgemm_family.py [--reps 5] [--loop N]
--loop N: just launch the 10 GEMMs N times (for rocprofv3 --pmc passes; dispatch i is shape i % 10)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402

SHAPES = ["ffn1_down_fwd", "ffn2_down_fwd", "out_fwd", "pw2_fwd", "ffn1_up_dgrad", "ffn2_up_dgrad", "qkv_dgrad",
          "out_dgrad", "pw1_dgrad", "pw2_dgrad"]


def build(M=32 * 373, d=512, F=2048):
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)

    def rn(*s, dt=bf, sc=1.0):
        return (torch.randn(*s, device="cuda", generator=g) * sc).to(dt)
    x2048 = rn(M, F)
    x512 = rn(M, d)
    dqkv = rn(M, 3 * d)
    da1024 = rn(M, 2 * d)
    res = rn(M, d, dt=torch.float32)
    w_dn = rn(d, F, sc=0.05)
    w_o = rn(d, d, sc=0.05)
    w_up_t = rn(d, F, sc=0.05)          # K-major copies (CastTBatch): (K, N) = W^T of (N, K) weights
    w_qkv_t = rn(d, 3 * d, sc=0.05)
    w_pw1_t = rn(d, 2 * d, sc=0.05)
    b = rn(d, dt=torch.float32)
    y32 = torch.empty(M, d, device="cuda", dtype=torch.float32)
    dx = torch.empty(M, d, device="cuda", dtype=bf)
    fl2048, fl512 = 2.0 * M * d * F, 2.0 * M * d * d
    cases = [
        (fl2048, lambda: ops.linear(x2048, w_dn, b, out=y32, drop_p=0.1, seed=2, out_scale=0.5, residual=res)),
        (fl2048, lambda: ops.linear(x2048, w_dn, b, out=y32, drop_p=0.1, seed=3, out_scale=0.5, residual=res)),
        (fl512, lambda: ops.linear(x512, w_o, b, out=y32, drop_p=0.1, seed=4, residual=res)),
        (fl512, lambda: ops.linear(x512, w_o, b, out=y32, drop_p=0.1, seed=5, residual=res)),
        (fl2048, lambda: ops.gemm(x2048, w_up_t, dx, M, d, F, lda=F, ldb=F)),
        (fl2048, lambda: ops.gemm(x2048, w_up_t, dx, M, d, F, lda=F, ldb=F)),
        (3 * fl512, lambda: ops.gemm(dqkv, w_qkv_t, dx, M, d, 3 * d, lda=3 * d, ldb=3 * d)),
        (fl512, lambda: ops.gemm(x512, w_o, dx, M, d, d)),
        (2 * fl512, lambda: ops.gemm(da1024, w_pw1_t, dx, M, d, 2 * d, lda=2 * d, ldb=2 * d)),
        (fl512, lambda: ops.gemm(x512, w_o, dx, M, d, d)),
    ]
    return cases


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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--loop", type=int, default=0)
    ap.add_argument("--mode", type=int, default=None)
    a = ap.parse_args()
    if a.mode is not None:
        from nn_conformer_for_speech_recognition_amd import _lib
        _lib.call("cfm_gemm_set_mode", a.mode)
    cases = build()
    if a.loop:
        for _ in range(a.loop):
            for _, fn in cases:
                fn()
        torch.cuda.synchronize()
        print("launched", a.loop, "x", len(cases))
        return
    ts = {k: [] for k in SHAPES}
    for _ in range(a.reps):
        for k, (fl, fn) in zip(SHAPES, cases):
            ts[k].append(timeit(fn))
    out, tot_t, tot_f = {}, 0.0, 0.0
    for k, (fl, _) in zip(SHAPES, cases):
        t = sorted(ts[k])[len(ts[k]) // 2]
        out[k] = round(t, 2)
        tot_t += t
        tot_f += fl
        print(f"{k:16s} {t:8.2f} us {fl / t / 1e6:7.0f} TF/s")
    print(f"{'layer total':16s} {tot_t:8.2f} us {tot_f / tot_t / 1e6:7.0f} TF/s = {tot_f / tot_t / 1e6 / 2500:.3f} of "
          f"bf16 peak; x17 layers = {17 * tot_t / 1e3:.2f} ms/step")
    print("DGEMM " + json.dumps({"lib": os.environ.get("CFM_LIB", "default"), "us": out, "layer_us": round(tot_t, 2),
                                 "tflops": round(tot_f / tot_t / 1e6, 1)}))


if __name__ == "__main__":
    main()
