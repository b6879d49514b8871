import torch, sys
sys.path.insert(0, '.')
from nn_conformer_for_speech_recognition_amd import ops, _lib
M, K = 11936, 512
g = torch.Generator(device='cuda').manual_seed(0)
x = torch.randn(M, K, device='cuda', generator=g).bfloat16()
for N in (1024, 1536, 2048):
    w = (torch.randn(N, K, device='cuda', generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device='cuda', generator=g)
    outs = []
    for m in (3, 3 | 2097152):
        _lib.call("cfm_gemm_set_mode", m)
        y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        pre = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        ops.linear(x, w, b, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=3, out=y)
        y2 = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        ops.linear(x, w, b, out=y2)
        torch.cuda.synchronize()
        outs.append((y.clone(), pre.clone(), y2.clone()))
    _lib.call("cfm_gemm_set_mode", 3)
    print(N, [torch.equal(a, c) for a, c in zip(*outs)])
