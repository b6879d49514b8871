"""A/B of the grouped weight-gradient launch variants (cfm_gemm_set_mode bits 8-9) on one layer's or
17 layers' worth of encoder weight-gradient GEMMs (M = 11,936 tokens)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402

M = 32 * 373
layer = [(2048, 512), (512, 2048), (1536, 512), (512, 512), (1024, 512), (512, 512), (2048, 512), (512, 2048)]
for nl in (1, 17):
    ops_ = [(torch.randn(M, N, device="cuda", dtype=torch.bfloat16), torch.randn(M, K, device="cuda", dtype=torch.bfloat16))
            for _ in range(nl) for (N, K) in layer]
    fl = sum(2.0 * M * d.shape[1] * x.shape[1] for d, x in ops_)
    grp = ops.WgradGroup()
    for mode in (3, 3 | 256, 3 | 768, 3, 3 | 768):   # bits 8-9: 0 256x256 (default), 1 256x128 BK32 x2, 3 256x128 BK64
        _lib.call("cfm_gemm_set_mode", mode)
        ts = []
        for it in range(6):
            for d, x in ops_:
                grp.add(d, x)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            grp.flush()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        t = sorted(ts[1:])[2]
        print(f"layers {nl:2d} mode {mode:4d}: {t:.3f} ms  {fl / t / 1e9:.0f} TF", flush=True)
    # the same GEMMs one by one (split-K + fused bias, today's side-stream path)
    _lib.call("cfm_gemm_set_mode", 3)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        s.record()
        for d, x in ops_:
            ops.linear_wgrad(d, x, bias_out=torch.empty(d.shape[1], device="cuda"))
        e.record()
        torch.cuda.synchronize()
    print(f"layers {nl:2d} per-GEMM split-K: {s.elapsed_time(e):.3f} ms  {fl / s.elapsed_time(e) / 1e9:.0f} TF", flush=True)
