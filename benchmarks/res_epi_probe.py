"""Price of the fp32 residual epilogue of the encoder's four residual GEMMs (FFN down K 2048, attention out /
pointwise-conv-2 K 512; M = 32 x 375, N = 512): the fused form (fp32 residual in, fp32 out, dropout, out_scale) against
a bf16 'delta' output (bias + dropout + out_scale, no residual), and the LayerNorm that follows, plain and with the
residual add moved into it (cfm_layernorm_fwd_res, when the library has it).
    python benchmarks/res_epi_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402


def timeit(fn, n=50, warm=10):
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


M, N = 32 * 375, 512
bf = torch.bfloat16
g = torch.ones(N, device="cuda")
be = torch.zeros(N, device="cuda")
x = torch.randn(M, N, device="cuda")
for K in (2048, 512):
    h = torch.randn(M, K, device="cuda", dtype=bf)
    w = torch.randn(N, K, device="cuda", dtype=bf) * 0.03
    b = torch.randn(N, device="cuda")
    yf = torch.empty(M, N, device="cuda")
    yd = torch.empty(M, N, device="cuda", dtype=bf)
    rows = []
    for _ in range(3):
        t_res = timeit(lambda: ops.linear(h, w, b, drop_p=0.1, seed=1, out_scale=0.5, residual=x, out=yf))
        t_dlt = timeit(lambda: ops.linear(h, w, b, drop_p=0.1, seed=1, out_scale=0.5, out=yd))
        t_bias = timeit(lambda: ops.linear(h, w, b, out=yd))
        rows.append((t_res, t_dlt, t_bias))
    for r in rows:
        print(f"K {K:5d}: fp32 residual {r[0]:6.1f} us | bf16 delta (drop, scale) {r[1]:6.1f} us | bf16 bias {r[2]:6.1f} us")
for _ in range(3):
    t_ln = timeit(lambda: ops.layernorm_fwd(x, g, be, 1e-5, out_dtype=bf))
    line = f"LayerNorm fwd fp32 x -> bf16: {t_ln:6.1f} us"
    if hasattr(ops, "layernorm_fwd_res"):
        t_lr = timeit(lambda: ops.layernorm_fwd_res(x, yd, g, be, 1e-5, out_dtype=bf))
        line += f" | with the residual add (x + bf16 delta -> fp32 x', bf16 y): {t_lr:6.1f} us"
    print(line)
