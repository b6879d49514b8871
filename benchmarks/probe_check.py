"""Cross-check of bench.py's in-kernel probe against HIP events over back-to-back launches (and,
run under rocprofv3 --kernel-trace, against the trace): FFN up-projection GEMM, bias+SiLU+dropout."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import KernelProbe  # noqa: E402
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402

M, N, K = 32 * 373, 2048, 512
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device="cuda")
pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
run = lambda: ops.linear(x, w, b, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=1, out=y)  # noqa: E731
for _ in range(10):
    run()
print("wallclock kHz", _lib.load().cfm_wallclock_khz())
probe = KernelProbe(lambda k, s, d: True, "cuda")
ops.PROBE = probe
probe.active = True
n = 40
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
s.record()
for _ in range(n):
    run()
e.record()
torch.cuda.synchronize()
print(f"events over {n} launches (incl. 2 probe kernels each): {s.elapsed_time(e) / n * 1e3:.1f} us/launch")
print(f"in-kernel probe: {probe.mean_ms()[0] * 1e3:.1f} us/launch over {probe.mean_ms()[1]}")
ops.PROBE = None
s.record()
for _ in range(n):
    run()
e.record()
torch.cuda.synchronize()
print(f"events over {n} plain launches: {s.elapsed_time(e) / n * 1e3:.1f} us/launch")
