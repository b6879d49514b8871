import time, torch
x = torch.randn(2048, 2048, device="cuda")
def work():
    y = x
    for _ in range(400):
        y = torch.tanh(y @ x * 1e-3)
    return y
work(); torch.cuda.synchronize()
gs = []
for k in range(2):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        work()
    gs.append(g)
torch.cuda.synchronize()
for mode in ("same", "alt"):
    ts = []
    t0 = time.perf_counter()
    for i in range(6):
        a = time.perf_counter()
        (gs[0] if mode == "same" else gs[i % 2]).replay()
        ts.append(round(1e3 * (time.perf_counter() - a), 2))
    torch.cuda.synchronize()
    print(mode, "replay host ms:", ts, "total ms", round(1e3 * (time.perf_counter() - t0), 1), flush=True)
