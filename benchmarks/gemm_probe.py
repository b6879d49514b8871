"""Launch only the roofline kernel of bench.py (FFN up-projection GEMM, M=11936 N=2048 K=512,
bf16, bias+SiLU epilogue, exactly as the encoder calls it) N times — for rocprofv3 --pmc passes
(FETCH_SIZE / WRITE_SIZE) whose per-dispatch counters then belong to that kernel alone.

    python benchmarks/gemm_probe.py [N] [--mode M] [--plain]
--mode: cfm_gemm_set_mode value (kernel variant A/B); --plain: bias only (no SiLU/pre/dropout)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="?", default=20)
ap.add_argument("--mode", type=int, default=None)
ap.add_argument("--plain", action="store_true")
ap.add_argument("--wgrad", action="store_true", help="the FFN W1 weight-gradient GEMM (split-K 8) instead")
a = ap.parse_args()
if a.mode is not None:
    _lib.call("cfm_gemm_set_mode", a.mode)

M, N, K = 32 * 373, 2048, 512
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
dyw = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(a.n):
    if a.wgrad:
        ops.linear_wgrad(dyw, x)
    elif a.plain:
        ops.linear(x, w, b, out=y)
    else:
        ops.linear(x, w, b, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=1, out=y)
torch.cuda.synchronize()
print("launched", a.n)
