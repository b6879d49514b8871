"""Micro-benchmarks of the hot kernels at the Conformer-L / 15 s shapes (B=32, T_enc=373,
M = 11,936 tokens).  Times each op with HIP events (median of N launches) and prints TFLOP/s or
GB/s.  Usage: python benchmarks/kernel_bench.py [--only gemm|attn|ln|conv]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402

DEV = "cuda"


def timeit(fn, n=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def bench_gemm():
    from nn_conformer_for_speech_recognition_amd import _lib
    _bench_gemm("warm-up pass (clocks ramp)")
    for mode, tag in ((0, "register-staged 128x128"), (1, "register-staged, 256x128 when wide"),
                      (2, "LDS-DMA pipeline"), (6, "LDS-DMA pipeline, 256x128 forced")):
        _lib.call("cfm_gemm_set_mode", mode)
        _bench_gemm(f"mode {mode}: {tag}")
    _lib.call("cfm_gemm_set_mode", 3)


def _bench_gemm(tag):
    M = 32 * 373
    bf = torch.bfloat16
    print(f"GEMM (bf16 operands, {tag}):")
    for (name, N, K) in [("ffn_up", 2048, 512), ("ffn_down", 512, 2048), ("qkv", 1536, 512), ("out/pw2", 512, 512),
                         ("pw1", 1024, 512)]:
        x = torch.randn(M, K, device=DEV, dtype=bf)
        w = torch.randn(N, K, device=DEV, dtype=bf) * 0.05
        b = torch.randn(N, device=DEV)
        fl = 2.0 * M * N * K
        y = torch.empty(M, N, device=DEV, dtype=bf)
        t = timeit(lambda: ops.linear(x, w, b, out=y))
        dy = torch.randn(M, N, device=DEV, dtype=bf)
        dx = torch.empty(M, K, device=DEV, dtype=bf)
        t2 = timeit(lambda: ops.linear_dgrad(dy, w, out=dx))
        t3 = timeit(lambda: ops.linear_wgrad(dy, x))
        print(f"  {name:9s} M={M} N={N} K={K}: fwd {t*1e3:7.1f}us {fl/t/1e9:6.0f} TF | dgrad {t2*1e3:7.1f}us "
              f"{fl/t2/1e9:6.0f} TF | wgrad {t3*1e3:7.1f}us {fl/t3/1e9:6.0f} TF")


def bench_attn():
    B, T, H, dk = 32, 373, 8, 64
    qkv = torch.randn(B * T, 3 * H * dk, device=DEV, dtype=torch.bfloat16)
    lens = torch.full((B,), T, dtype=torch.int32, device=DEV)
    fl = 4.0 * B * H * T * T * dk
    from nn_conformer_for_speech_recognition_amd import _lib
    for mode, p in ((0, 0.0), (0, 0.1), (8, 0.0), (8, 0.1), (2, 0.0), (4, 0.0)):
        _lib.call("cfm_attn_set_mode", mode)
        o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=p, seed=3)
        t = timeit(lambda: ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=p, seed=3))
        do = torch.randn_like(o)
        t2 = timeit(lambda: ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=p, seed=3))
        print(f"attention mode={mode} B={B} T={T} H={H} dk={dk} p={p}: fwd {t*1e3:.1f}us {fl/t/1e9:.0f} TF | bwd "
              f"{t2*1e3:.1f}us {2.5*fl/t2/1e9:.0f} TF")


def bench_ln():
    M, D = 32 * 373, 512
    x = torch.randn(M, D, device=DEV)
    g = torch.ones(D, device=DEV)
    bt = torch.zeros(D, device=DEV)
    y, mu, rs = ops.layernorm_fwd(x, g, bt, out_dtype=torch.bfloat16)
    t = timeit(lambda: ops.layernorm_fwd(x, g, bt, out_dtype=torch.bfloat16))
    dy = torch.randn(M, D, device=DEV, dtype=torch.bfloat16)
    t2 = timeit(lambda: ops.layernorm_bwd(dy, x, g, mu, rs, dres=x))
    print(f"layernorm M={M} D={D}: fwd {t*1e3:.1f}us {M*D*6/t/1e6:.0f} GB/s | bwd {t2*1e3:.1f}us "
          f"{M*D*14/t2/1e6:.0f} GB/s")


def bench_conv():
    B, T, C, K = 32, 373, 512, 31
    a = torch.randn(B * T, 2 * C, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(C, K, device=DEV) * 0.1
    bias = torch.randn(C, device=DEV)
    ws = ops.convmod_ws(B, T, C, K, a.device)
    t = timeit(lambda: ops.glu_dwconv_fwd(a, w, bias, B, T, C, K, ws))
    dy = torch.randn(B * T, C, device=DEV)
    t2 = timeit(lambda: ops.glu_dwconv_bwd(dy, a, w, B, T, C, K, ws, torch.bfloat16))
    nb = B * T * C
    print(f"glu_dwconv B={B} T={T} C={C} K={K}: fwd {t*1e3:.1f}us {nb*(4+4)/t/1e6:.0f} GB/s | bwd {t2*1e3:.1f}us "
          f"{nb*(4+4+4)/t2/1e6:.0f} GB/s")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    for name, fn in (("gemm", bench_gemm), ("attn", bench_attn), ("ln", bench_ln), ("conv", bench_conv)):
        if a.only in (None, name):
            fn()




