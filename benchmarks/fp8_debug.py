"""Debug aid: compare cfm_quant_fp8 with torch's float8_e4m3fn conversion element by element."""
import sys
import torch
sys.path.insert(0, '/root/repo')
from nn_conformer_for_speech_recognition_amd import ops
for dt in (torch.float32, torch.bfloat16):
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(1000, 264, generator=g) * 3).to(dt)
    x[3, 7] = -17.25
    y, sc = ops.quant_fp8(x.cuda())
    amax = x.float().abs().max()
    v = x.float() * (448.0 / amax)
    ref = v.to(torch.float8_e4m3fn)
    a, b = y.cpu().view(torch.uint8), ref.view(torch.uint8)
    bad = (a != b).nonzero()
    print(dt, "amax", amax.item(), "sc", sc.item(), "mismatches", bad.shape[0])
    for i in range(min(8, bad.shape[0])):
        r, c = bad[i].tolist()
        print("  ", r, c, v[r, c].item(), "gpu", a[r, c].item(), y.cpu()[r, c].float().item(), "torch", b[r, c].item(),
              ref[r, c].float().item())
