"""The 96-row two-per-CU GEMM variant (cfm_gemm_set_mode bit 18) vs the default 192-row tiles on the encoder's
d-wide GEMMs (M 11,936, N 512, K 512 / 2048, fp32 out + residual + dropout, bf16 out): bitwise comparison."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402

M, d = 32 * 373, 512
g = torch.Generator().manual_seed(0)
for K in (512, 2048):
    x = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
    w = (0.05 * torch.randn(d, K, generator=g)).to("cuda", torch.bfloat16)
    b = torch.randn(d, generator=g).cuda()
    res = torch.randn(M, d, generator=g).cuda()
    outs = []
    for mode in (3, 3 | 262144):
        _lib.call("cfm_gemm_set_mode", mode)
        y = ops.linear(x, w, b, out_dtype=torch.float32, drop_p=0.1, seed=3, out_scale=0.5, residual=res)
        z = ops.linear(x, w, b)
        torch.cuda.synchronize()
        outs.append((y.clone(), z.clone()))
    _lib.call("cfm_gemm_set_mode", 3)
    ref = (x.float() @ w.float().t() + b)
    print(f"K={K}: fp32+res bitwise {torch.equal(outs[0][0], outs[1][0])} max|d| {(outs[0][0]-outs[1][0]).abs().max().item():.3g}; "
          f"bf16 bitwise {torch.equal(outs[0][1], outs[1][1])}; v96 vs fp32 ref rel {((outs[1][1].float()-ref).norm()/ref.norm()).item():.2e}")
