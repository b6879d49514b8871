"""Utterance-batch data parallelism: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) across xGMI.  The reference is single-device; this is the one
exchange step the build adds: an all-reduce (average) of every gradient after backward.

Gradients are packed into a few large flat buckets (default 64 MB) so RCCL runs long, per-link
bandwidth-bound rings instead of hundreds of small latency-bound calls.  Equal per-rank batches
make the averaged per-rank CTC-mean gradients equal to the global-batch mean gradient.
BatchNorm statistics stay per-replica (as in DDP without SyncBN).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the process group from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, local


def broadcast_parameters(module, src=0):
    """Rank src's initial weights (and buffers) everywhere."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


class GradAllReducer:
    """Average the gradients of `params` over the default process group in flat buckets."""

    def __init__(self, params, bucket_bytes=64 << 20):
        self.params = [p for p in params if p.requires_grad]
        self.buckets = []
        cur, size = [], 0
        for p in self.params:
            nbytes = p.numel() * 4
            if cur and size + nbytes > bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self._flat = [None] * len(self.buckets)

    def allreduce(self):
        if not (dist.is_available() and dist.is_initialized()):
            return
        world = dist.get_world_size()
        if world == 1:
            return
        for i, bucket in enumerate(self.buckets):
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            n = sum(g.numel() for g in grads)
            flat = self._flat[i]
            if flat is None or flat.numel() != n or flat.device != grads[0].device:
                flat = torch.empty(n, device=grads[0].device, dtype=torch.float32)
                self._flat[i] = flat
            off = 0
            for g in grads:
                flat[off:off + g.numel()].copy_(g.reshape(-1))
                off += g.numel()
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
            flat.mul_(1.0 / world)
            off = 0
            for p, g in zip(bucket, grads):
                if p.grad is None:
                    p.grad = g
                p.grad.copy_(flat[off:off + g.numel()].view_as(p.grad))
                off += g.numel()


def global_batch_slice(global_batch, rank, world):
    """Contiguous slice [lo, hi) of the global utterance batch owned by `rank`."""
    per = global_batch // world
    return rank * per, (rank + 1) * per
