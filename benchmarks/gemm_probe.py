"""Launch only the roofline kernel of bench.py (FFN up-projection GEMM, M=11936 N=2048 K=512,
bf16, bias+SiLU epilogue, exactly as the encoder calls it) N times — for rocprofv3 --pmc passes
(FETCH_SIZE / WRITE_SIZE) whose per-dispatch counters then belong to that kernel alone."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402

M, N, K = 32 * 373, 2048, 512
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(n):
    ops.linear(x, w, b, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=1, out=y)
torch.cuda.synchronize()
print("launched", n)
