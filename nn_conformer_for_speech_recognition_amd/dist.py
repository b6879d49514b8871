"""Utterance-batch data parallelism: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) across xGMI.  The reference is single-device; this is the one
exchange step the build adds: an all-reduce (average) of every gradient after backward.

Gradients live in a few large flat buckets (the Conformer's grouped weight gradients are WRITTEN into
them by the grouped launch: no copies) so RCCL runs long, per-link bandwidth-bound rings instead of
hundreds of small latency-bound calls, optionally overlapped with the rest of the backward (eager).
Equal per-rank batches make the averaged per-rank CTC-mean gradients equal to the global-batch mean
gradient.  BatchNorm statistics stay per-replica (as in DDP without SyncBN); with BN in eval mode the
averaged gradients equal the single-process gradients of the global batch (tests/test_gpu_dist.py).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the process group from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("CFM_SHARE_DEVICE"):
        local = 0          # rehearsal of N ranks on one GPU (gloo): every rank on device 0
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = os.environ.get("CFM_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
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


# _PNAMES indices of the weights whose gradients (with the following bias) the grouped weight-gradient
# launch produces -- the bulk of every Conformer layer's gradient bytes
_GROUPED_W = (2, 4, 8, 10, 14, 20, 24, 26)


def _avg_op():
    """ReduceOp.AVG where the backend has it (RCCL/NCCL); gloo: SUM then a scale."""
    return dist.ReduceOp.AVG if dist.get_backend() == "nccl" else None


class GradAllReducer:
    """Average the gradients of `params` over the default process group.

    Layout: each Conformer layer's grouped weight/bias gradients live in flat fp32 BUCKETS (one per
    chunk of `chunk_layers` layers, in backward order); attach(conformer) hands the layers views of them,
    so the grouped weight-gradient launch writes straight into the bucket and autograd adopts the views
    as .grad (no copy-in / copy-out).  Every other gradient (LayerNorm / BatchNorm / depthwise-conv /
    rel-pos / front-end / head) goes through one small flat tail bucket (copy in, reduce, copy out).

    Overlap: with overlap=True (eager backward) the Conformer flushes its grouped launch at each chunk
    boundary and calls back here; the chunk's bucket all-reduce is then issued asynchronously (RCCL runs
    it on its own stream, ordered after the flush) while the lower layers' backward continues.
    allreduce() issues whatever is left (all buckets when not overlapping) and waits for everything.
    Inside a captured HIP graph use overlap=False and call allreduce() after the replay."""

    def __init__(self, params, bucket_bytes=64 << 20, model=None, chunk_layers=4, overlap=False):
        self.params = [p for p in params if p.requires_grad]
        self.bucket_bytes = bucket_bytes
        self.overlap = overlap
        self.flat = []            # chunk buckets: (flat tensor, lo_layer, hi_layer)
        self.pending = []         # async work handles of this step
        self.launched = set()
        self.routed = set()       # Conformer layers whose grouped gradients all landed in the buckets
        self._no_sync = False
        self.conformer = None
        owned = set()
        if model is not None:
            from .conformer import Conformer
            conf = [m for m in model.modules() if isinstance(m, Conformer)]
            if conf and conf[0].compute_dtype == torch.bfloat16:
                owned = self._attach(conf[0], chunk_layers)
        self.tail = [p for p in self.params if id(p) not in owned]
        self.buckets = []         # tail buckets of params (legacy name: lists of params)
        cur, size = [], 0
        for p in self.tail:
            nbytes = p.numel() * 4
            if cur and size + nbytes > bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self._tail_flat = [None] * len(self.buckets)

    # ------------------------------------------------------------------------------ Conformer buckets
    def _attach(self, conf, chunk_layers):
        layers = list(conf.conformer_layers)
        n = len(layers)
        dev = next(conf.parameters()).device
        owned = set()
        dest = [dict() for _ in range(n)]
        # chunks in backward order: layers [n-c, n), [n-2c, n-c), ...
        hi = n
        flush = set()
        while hi > 0:
            lo = max(0, hi - chunk_layers)
            views = []
            total = 0
            for li in range(lo, hi):
                ps = layers[li].params()
                for wi in _GROUPED_W:
                    w, b = ps[wi], ps[wi + 1]
                    N = w.shape[0]
                    K = w.numel() // N
                    views.append((li, wi, N, K, total, total + (N * K + 63) // 64 * 64))
                    total += (N * K + 63) // 64 * 64 + (N + 63) // 64 * 64
                    owned.add(id(w))
                    owned.add(id(b))
            flat = torch.zeros(max(total, 1), device=dev, dtype=torch.float32)
            for li, wi, N, K, ow, ob in views:
                dest[li][wi] = (flat[ow:ow + N * K].view(N, K), flat[ob:ob + N])
            self.flat.append((flat, lo, hi))
            flush.add(lo)
            hi = lo
        conf.grad_dest = dest
        self.conformer = conf
        if self.overlap:
            conf.flush_layers = frozenset(flush)
            conf.on_flushed = self._on_flushed
            conf.on_routed = self._on_routed
        return owned

    def _world(self):
        if not (dist.is_available() and dist.is_initialized()):
            return 1
        return dist.get_world_size()

    def _reduce(self, t, async_op):
        op = _avg_op()
        if op is not None:
            return dist.all_reduce(t, op=op, async_op=async_op)
        w = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)
        if async_op:
            w.wait()
        t.mul_(1.0 / dist.get_world_size())
        return None

    def _on_flushed(self, layer_index):
        """Called by the Conformer right after it flushed the grouped launch at `layer_index`: every chunk
        whose layers are all >= layer_index is final -> issue its all-reduce now (async).  Only chunks whose
        every grouped weight/bias gradient was WRITTEN into its bucket view by this backward's grouped launch
        (on_routed) qualify: a layer that accumulated into an existing .grad, or skipped the grouped launch
        (gradient hooks, unsupported operand shapes), finishes its gradients through AccumulateGrad AFTER
        this call, so its chunk waits for allreduce().  Nothing launches under no_sync()."""
        if self._world() == 1 or self._no_sync:
            return
        for i, (flat, lo, hi) in enumerate(self.flat):
            if i in self.launched or lo < layer_index:
                continue
            if not all(li in self.routed for li in range(lo, hi)):
                continue
            self.launched.add(i)
            w = self._reduce(flat, True)
            if w is not None:
                self.pending.append(w)

    def _on_routed(self, layer_index):
        """The Conformer's layer `layer_index` routed all its grouped gradients into the bucket views."""
        self.routed.add(layer_index)

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation over micro-batches (DDP's no_sync): backward passes inside the context issue
        no bucket all-reduce; the allreduce() after the last micro-batch reduces the accumulated gradients."""
        prev = self._no_sync
        self._no_sync = True
        try:
            yield
        finally:
            self._no_sync = prev
            self.routed = set()

    def _chunk_views(self, chunk):
        """(param, bucket view) pairs of one chunk's grouped gradients."""
        _, lo, hi = self.flat[chunk]
        out = []
        for li in range(lo, hi):
            ps = self.conformer.conformer_layers[li].params()
            for wi, (dw, db) in self.conformer.grad_dest[li].items():
                out += [(ps[wi], dw), (ps[wi + 1], db)]
        return out

    def _adopt(self, chunk, copy):
        """Make every grouped gradient of `chunk` its bucket view.  copy=True (chunk not yet reduced): a
        gradient living elsewhere is copied in first.  copy=False (chunk reduced during backward, only from
        fully routed layers): the bucket already holds the reduced gradient, so .grad is just re-pointed."""
        for p, v in self._chunk_views(chunk):
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                if copy:
                    v.copy_(p.grad.reshape(v.shape))
                p.grad = v.view(p.shape)

    def allreduce(self):
        if self._world() == 1:
            self.launched.clear()
            self.routed = set()
            return
        if self.conformer is not None:
            for i in range(len(self.flat)):
                if i not in self.launched:
                    self._adopt(i, copy=True)      # before any of those chunks' reductions starts
        for i, (flat, lo, hi) in enumerate(self.flat):
            if i not in self.launched:
                w = self._reduce(flat, True)
                if w is not None:
                    self.pending.append(w)
        for i, bucket in enumerate(self.buckets):
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            n = sum(g.numel() for g in grads)
            flat = self._tail_flat[i]
            if flat is None or flat.numel() != n or flat.device != grads[0].device:
                flat = torch.empty(n, device=grads[0].device, dtype=torch.float32)
                self._tail_flat[i] = flat
            off = 0
            for g in grads:
                flat[off:off + g.numel()].copy_(g.reshape(-1))
                off += g.numel()
            self._reduce(flat, False)
            off = 0
            for p, g in zip(bucket, grads):
                if p.grad is None:
                    p.grad = g
                p.grad.copy_(flat[off:off + g.numel()].view_as(p.grad))
                off += g.numel()
        for w in self.pending:
            w.wait()
        if self.conformer is not None:
            for i in self.launched:
                self._adopt(i, copy=False)
        self.pending = []
        self.launched = set()
        self.routed = set()


def global_batch_slice(global_batch, rank, world):
    """Contiguous slice [lo, hi) of the global utterance batch owned by `rank`."""
    per = global_batch // world
    return rank * per, (rank + 1) * per
