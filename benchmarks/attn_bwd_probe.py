"""Attention backward kernels at Conformer-L / 15 s (B 32, T 373, H 8, dk 64) for rocprofv3 --stats:
dK/dV wave kernel (mode 0) and the four-wave head kernel (mode 8), dropout 0.1 and 0; N launches each.
Usage: rocprofv3 --kernel-trace --stats -- python3 benchmarks/attn_bwd_probe.py [N] [modes] [drop ps]
(modes / ps comma-separated, default "0,8" and "0.1,0.0")"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, T, H, dk = 32, 373, 8, 64
g = torch.Generator().manual_seed(0)
qkv = torch.randn(B * T, 3 * H * dk, generator=g).to("cuda", torch.bfloat16)
do = torch.randn(B * T, H * dk, generator=g).to("cuda", torch.bfloat16)
lens = torch.tensor([T - (i * 7) % 90 for i in range(B)], dtype=torch.int32, device="cuda")
MODES = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,8").split(",")]
PS = [float(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0.1,0.0").split(",")]
for mode in MODES:
    for p in PS:
        _lib.call("cfm_attn_set_mode", mode)
        o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=p, seed=3)
        for _ in range(N):
            ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=p, seed=3)
        torch.cuda.synchronize()
        print(f"mode {mode} p {p} done", flush=True)
_lib.call("cfm_attn_set_mode", 0)
