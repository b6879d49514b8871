"""Dump the rel-pos attention forward / backward outputs (L60 shape, ragged lengths, dropout 0.1) of the libcfm
build CFM_LIB selects, or compare two dumps bit for bit -- for layout-only kernel changes that must not move a bit.
    CFM_LIB=a.so python benchmarks/rel_dump.py dump OUT.pt ; python benchmarks/rel_dump.py cmp A.pt B.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(out):
    from nn_conformer_for_speech_recognition_amd import ops
    B, T, H, dk = 8, 1498, 8, 64
    g = torch.Generator().manual_seed(1)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to("cuda", torch.bfloat16)
    pos = (0.5 * torch.randn(2 * T - 1, H * dk, generator=g)).to("cuda", torch.bfloat16)
    pu = (0.3 * torch.randn(H * dk, generator=g)).cuda()
    pv = (0.3 * torch.randn(H * dk, generator=g)).cuda()
    do = torch.randn(B * T, H * dk, generator=g).to("cuda", torch.bfloat16)
    lens = torch.tensor([T, T - 1, 1201, 1100, 977, 640, 333, 65], dtype=torch.int32, device="cuda")
    res = {}
    for p in (0.0, 0.1):
        o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, pos, pu, pv, drop_p=p, seed=5)
        grads = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, pos, pu, pv, drop_p=p, seed=5)
        res[f"o{p}"] = o.cpu()
        for i, t in enumerate(grads if isinstance(grads, (tuple, list)) else (grads,)):
            if t is not None:
                res[f"g{p}_{i}"] = t.cpu()
    torch.cuda.synchronize()
    torch.save(res, out)
    print("dumped", out, sorted(res))


def cmp(a, b):
    A, Bd = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for k in sorted(A):
        same = torch.equal(A[k], Bd[k])
        bad += not same
        print(f"{k}: {'identical' if same else 'DIFFERS max %.3g' % (A[k].float() - Bd[k].float()).abs().max()}")
    print("BITEXACT" if bad == 0 else f"MISMATCH {bad}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    dump(sys.argv[2]) if sys.argv[1] == "dump" else cmp(sys.argv[2], sys.argv[3])
