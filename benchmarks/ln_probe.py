"""LayerNorm backward at the L15 shape as the step launches it (bf16 dy, fp32 x, residual gradient, fused
dropout-scaled bf16 g2): HIP-event timing over N launches.   python benchmarks/ln_probe.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
M, D = 32 * 373, 512
g = torch.Generator().manual_seed(0)
x = torch.randn(M, D, generator=g).cuda()
gam = (1 + 0.1 * torch.randn(D, generator=g)).cuda()
bt = torch.zeros(D, device="cuda")
y, mu, rs = ops.layernorm_fwd(x, gam, bt, out_dtype=torch.bfloat16)
dy = torch.randn(M, D, generator=g).to("cuda", torch.bfloat16)
dres = torch.randn(M, D, generator=g).cuda()
drop = (0.5, 0.1, 7, torch.bfloat16)
for _ in range(3):
    ops.layernorm_bwd(dy, x, gam, mu, rs, dres=dres, drop=drop)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(n):
    ops.layernorm_bwd(dy, x, gam, mu, rs, dres=dres, drop=drop)
e.record()
torch.cuda.synchronize()
print(f"layernorm bwd (+dres, +g2) {s.elapsed_time(e) / n * 1e3:.1f} us per call")
