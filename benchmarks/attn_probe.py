"""Attention forward timing experiments (cfm_attn_set_mode dbg bits) for rocprofv3 --stats:
mode 0 full, 2 staging only, 4 no epilogue stores; N launches each."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402

B, T, H, dk = 32, 373, 8, 64
qkv = torch.randn(B * T, 3 * H * dk, device="cuda", dtype=torch.bfloat16)
lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
for mode in (0, 2, 4, 0):
    _lib.call("cfm_attn_set_mode", mode)
    for _ in range(20):
        ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=3)
    torch.cuda.synchronize()
_lib.call("cfm_attn_set_mode", 0)
