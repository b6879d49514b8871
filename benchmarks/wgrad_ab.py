"""Weight-gradient GEMM layouts A/B: dW (N x K) = dY^T X over M = 11,936 tokens, as today (both operands
MN-major, tr16 reads) vs pre-transposed K-major operands, for several split-K counts."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402


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


M = 32 * 373
bf = torch.bfloat16
for name, N, K in [("ffn_w1", 2048, 512), ("ffn_w2", 512, 2048), ("qkv", 1536, 512), ("out", 512, 512), ("pw1", 1024, 512)]:
    dy = torch.randn(M, N, device="cuda", dtype=bf)
    x = torch.randn(M, K, device="cuda", dtype=bf)
    dyt, xt = dy.t().contiguous(), x.t().contiguous()
    fl = 2.0 * M * N * K
    row = []
    for split in (4, 8, 16):
        out = torch.empty(N, K, device="cuda")
        ws = torch.empty(split * N * K, device="cuda")
        t1 = timeit(lambda: ops.gemm(dy, x, out, N, K, M, a_kmajor=False, b_kmajor=False, lda=N, ldb=K,
                                     split_k=split, workspace=ws))
        t2 = timeit(lambda: ops.gemm(dyt, xt, out, N, K, M, a_kmajor=True, b_kmajor=True, lda=M, ldb=M,
                                     split_k=split, workspace=ws))
        row.append(f"split {split:2d}: MN {t1:6.1f}us ({fl/t1/1e6:4.0f}) KK {t2:6.1f}us ({fl/t2/1e6:4.0f})")
    print(f"{name:7s} N={N} K={K} | " + " | ".join(row), flush=True)
