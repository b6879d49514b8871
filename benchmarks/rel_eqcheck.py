"""Bit-identity of the rel-pos attention backward across cfm_attn_set_mode values (the first mode is compared
with the second and with the last):  python benchmarks/rel_eqcheck.py 0,MODE[,MODE2]"""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops
modes = [int(m) for m in sys.argv[1].split(',')]
for (B, T, H, lens) in [(2, 1498, 3, [1498, 1001]), (3, 373, 2, [373, 300, 41]), (2, 64, 1, [64, 1]), (9, 130, 2, [130] * 8 + [77])]:
    dk = 64
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to("cuda", torch.bfloat16)
    pos = (0.5 * torch.randn(2 * T - 1, H * dk, generator=g)).to("cuda", torch.bfloat16)
    pu = (0.3 * torch.randn(H * dk, generator=g)).cuda(); pv = (0.3 * torch.randn(H * dk, generator=g)).cuda()
    do = torch.randn(B * T, H * dk, generator=g).to("cuda", torch.bfloat16)
    ln = torch.tensor(lens, dtype=torch.int32, device="cuda")
    outs = []
    for m in modes:
        _lib.call("cfm_attn_set_mode", m)
        o, lse = ops.attn_fwd(qkv, ln, B, T, H, dk, pos, pu, pv, drop_p=0.1, seed=11)
        outs.append([t.clone() if torch.is_tensor(t) else t for t in ops.attn_bwd(qkv, o, do, lse, ln, B, T, H, dk, pos, pu, pv, drop_p=0.1, seed=11)])
    _lib.call("cfm_attn_set_mode", 0)
    diffs = [("%d:%s" % (i, "eq" if torch.equal(a, b) else "%.3g" % (a.float() - b.float()).abs().max().item()))
             for i, (a, b) in enumerate(zip(outs[0], outs[-1])) if torch.is_tensor(a)]
    rep = [torch.equal(a, b) for a, b in zip(outs[0], outs[1]) if torch.is_tensor(a)]
    print("EQ", B, T, H, "first-vs-last", diffs, "first-vs-second", rep)
