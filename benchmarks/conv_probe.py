"""Launch the conv-module kernels at the Conformer-L / 15 s shape (B 32, T 373, C 512, K 31) as the step does
(GLU + depthwise fwd, BN+SiLU fwd, BN sums + BN-folded depthwise backward) N times: timing with HIP events
and a target for rocprofv3 --pmc passes (benchmarks/pmc_kernels.sh).
    python benchmarks/conv_probe.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, T, C, K = 32, 373, 512, 31
g = torch.Generator().manual_seed(0)
a = torch.randn(B * T, 2 * C, generator=g).to("cuda", torch.bfloat16)
w = (0.1 * torch.randn(C, K, generator=g)).cuda()
bias = (0.1 * torch.randn(C, generator=g)).cuda()
gamma = (1 + 0.1 * torch.randn(C, generator=g)).cuda()
beta = (0.1 * torch.randn(C, generator=g)).cuda()
rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
dz = torch.randn(B * T, C, generator=g).to("cuda", torch.bfloat16)
ws = torch.empty(64 << 20, device="cuda", dtype=torch.uint8)


def step():
    y = ops.glu_dwconv_fwd(a, w, bias, B, T, C, K, ws)
    z, mean, inv = ops.bn_silu_fwd(y, gamma, beta, rm, rv, 0.1, 1e-5, True, B, T, C, ws, torch.bfloat16)
    return ops.bn_silu_glu_dwconv_bwd(dz, y, gamma, beta, mean, inv, True, a, w, B, T, C, K, ws, torch.bfloat16)


step()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(n):
    step()
e.record()
torch.cuda.synchronize()
print(f"conv module fwd+bwd kernels {s.elapsed_time(e) / n * 1e3:.1f} us per call")
