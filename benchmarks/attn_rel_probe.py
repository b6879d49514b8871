"""Launch the rel-pos attention kernels at the L60 shape (B 8, T 1498, H 8, dk 64) N times, for rocprofv3
--pmc passes (benchmarks/pmc_kernels.sh) and quick timing.   python benchmarks/attn_rel_probe.py [N] [--none]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="?", default=5)
ap.add_argument("--none", action="store_true", help="no relative positions (tiled kernels)")
ap.add_argument("--l15", action="store_true", help="the L15 shape (B 32, T 373: whole-head kernels when --none)")
ap.add_argument("--p", type=float, default=0.1, help="attention dropout")
ap.add_argument("--mode", type=int, default=0, help="cfm_attn_set_mode value (A/B)")
ap.add_argument("--dpos-f32", action="store_true", help="fp32 dpos (the step writes bf16 dpos for bf16 rel-pos)")
a = ap.parse_args()
if a.mode:
    from nn_conformer_for_speech_recognition_amd import _lib  # noqa: E402
    _lib.call("cfm_attn_set_mode", a.mode)
B, T, H, dk = (32, 373, 8, 64) if a.l15 else (8, 1498, 8, 64)
g = torch.Generator().manual_seed(0)
qkv = torch.randn(B * T, 3 * H * dk, generator=g).to("cuda", torch.bfloat16)
pos = None if a.none else (0.5 * torch.randn(2 * T - 1, H * dk, generator=g)).to("cuda", torch.bfloat16)
pu = None if a.none else (0.3 * torch.randn(H * dk, generator=g)).cuda()
pv = None if a.none else (0.3 * torch.randn(H * dk, generator=g)).cuda()
do = torch.randn(B * T, H * dk, generator=g).to("cuda", torch.bfloat16)
lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for i in range(a.n + 1):
    if i == 1:
        torch.cuda.synchronize()
        s.record()
    o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, pos, pu, pv, drop_p=a.p, seed=3)
    ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, pos, pu, pv, drop_p=a.p, seed=3,
                 dpos_dtype=torch.float32 if (a.dpos_f32 or a.none) else torch.bfloat16)
e.record()
torch.cuda.synchronize()
print(f"fwd+bwd {s.elapsed_time(e) / max(a.n, 1) * 1e3:.1f} us per call")
