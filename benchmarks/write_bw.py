import torch
def t(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e)/n*1e3
for mb in (49, 98, 196):
    x=torch.empty(mb*1024*1024//2, dtype=torch.bfloat16, device='cuda')
    y=torch.empty_like(x)
    us=t(lambda: x.fill_(1.0)); print(f"fill {mb} MB: {us:.1f} us  {mb*1.048576/us:.2f} TB/s")
    us=t(lambda: y.copy_(x)); print(f"copy {mb} MB: {us:.1f} us  {2*mb*1.048576/us:.2f} TB/s (r+w)")
