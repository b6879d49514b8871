"""LayerNorm forward / backward (+ residual gradient, fused dropout-scaled bf16 g2) at the encoder widths
(144 / 256 / 512) and the 32 x 373-frame batch: HIP-event time per call and the bytes-per-second it implies."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops
def t(fn, n=50):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3
for D in (144, 256, 512):
    M = 32 * 373
    g = torch.Generator().manual_seed(0)
    x = torch.randn(M, D, generator=g).cuda()
    gam = (1 + 0.1 * torch.randn(D, generator=g)).cuda(); bt = torch.zeros(D, device="cuda")
    y, mu, rs = ops.layernorm_fwd(x, gam, bt, out_dtype=torch.bfloat16)
    dy = torch.randn(M, D, generator=g).to("cuda", torch.bfloat16)
    dres = torch.randn(M, D, generator=g).cuda()
    drop = (0.5, 0.1, 7, torch.bfloat16)
    tb = t(lambda: ops.layernorm_bwd(dy, x, gam, mu, rs, dres=dres, drop=drop))
    tf = t(lambda: ops.layernorm_fwd(x, gam, bt, out_dtype=torch.bfloat16))
    bb = M * D * (2 + 4 + 4 + 4 + 2); bf = M * D * (4 + 2)
    print(f"D {D}: bwd {tb:6.1f} us ({bb / tb / 1e6:.2f} TB/s)  fwd {tf:6.1f} us ({bf / tf / 1e6:.2f} TB/s)")
