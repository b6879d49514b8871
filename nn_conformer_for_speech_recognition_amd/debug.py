"""Numerics tripwire for debugging (off by default): CFM_NANCHECK=1 makes check() synchronise and report
the first tensors of a step that hold NaN/Inf, by name, in launch order.  Skipped inside HIP-graph capture
(the check needs a host read).  Used by benchmarks/nan_hunt.py together with bench.py --poison (every
torch.empty NaN-filled), which turns a read of never-written memory into a named non-finite tensor."""
from __future__ import annotations

import os

import torch

ENABLED = bool(os.environ.get("CFM_NANCHECK"))
LIMIT = int(os.environ.get("CFM_NANCHECK_LIMIT", "40"))
HITS = []


def check(name, *tensors):
    if not ENABLED or torch.cuda.is_current_stream_capturing():
        return
    for i, t in enumerate(tensors):
        if t is None or not torch.is_tensor(t) or not t.is_floating_point():
            continue
        if not bool(torch.isfinite(t.float() if t.dtype == torch.float8_e4m3fn else t).all()):
            HITS.append(f"{name}[{i}]")
            if len(HITS) <= LIMIT:
                bad = (~torch.isfinite(t.float())).sum().item()
                print(f"[nancheck] non-finite: {name}[{i}] shape={tuple(t.shape)} dtype={t.dtype} "
                      f"count={bad}/{t.numel()}", flush=True)


def reset():
    HITS.clear()
