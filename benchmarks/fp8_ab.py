"""A/B: fp8 (e4m3, block-scaled MFMA) vs bf16 forward GEMMs of the encoder shapes, GEMM alone and with
the per-tensor quantisation of the activation operand.   python benchmarks/fp8_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402


def timeit(fn, n=30, warm=5):
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


M = 8 * 1498
for name, N, K, silu in [("ffn_up", 2048, 512, True), ("ffn_down", 512, 2048, False), ("qkv", 1536, 512, False),
                         ("out", 512, 512, False)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda") * 0.05
    wb = w.to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if silu else None
    xq, sx = ops.quant_fp8(x)
    wq, sw = ops.quant_fp8(w)
    kw = dict(act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=1) if silu else {}
    t_bf = timeit(lambda: ops.linear(x, wb, b, **kw))
    t_f8 = timeit(lambda: ops.linear(xq, wq, b, x_scale=sx, w_scale=sw, **kw))
    t_q = timeit(lambda: ops.quant_fp8(x, out=xq, inv_scale=sx))
    fl = 2.0 * M * N * K
    print(f"{name:8s} M={M} N={N:5d} K={K:5d}  bf16 {t_bf:7.1f} us ({fl / t_bf / 1e6:5.0f} TF/s)   "
          f"fp8 {t_f8:7.1f} us ({fl / t_f8 / 1e6:5.0f} TF/s)   quant(x) {t_q:6.1f} us")
