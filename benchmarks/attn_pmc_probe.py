"""The L15 attention kernels as the step runs them (B 32, T 373, 8 heads, dk 64, dropout 0.1, default kernel
selection), n forward + backward pairs: the command benchmarks/attn_pmc.sh profiles with rocprofv3 --pmc.
    python benchmarks/attn_pmc_probe.py [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    B, T, H, dk = 32, 373, 8, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * T, 3 * H * dk, device="cuda", generator=g).to(torch.bfloat16)
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    do = torch.randn(B * T, H * dk, device="cuda", generator=g).to(torch.bfloat16)
    for _ in range(n):
        o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=3)
        ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=0.1, seed=3)
    torch.cuda.synchronize()
    print("attn probe done", n)


if __name__ == "__main__":
    main()
