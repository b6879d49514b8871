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
    HIP graphs: SegmentedStepGraph captures the step as a chain of graphs cut at those same flush points and
    issues each finished chunk's all-reduce between two replays (the collectives themselves are never
    captured); a single captured graph (overlap=False) reduces everything in allreduce() after the replay.

    grad_dtype=torch.bfloat16: the buckets are reduced through bf16 copies (half the xGMI bytes; each rank's
    fp32 bucket is cast down, summed/averaged in bf16 by the collective, cast back into the fp32 bucket).
    The optimizer still reads fp32 gradients and updates fp32 master weights."""

    def __init__(self, params, bucket_bytes=64 << 20, model=None, chunk_layers=4, overlap=False,
                 grad_dtype=torch.float32):
        if grad_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"grad_dtype must be float32 or bfloat16, got {grad_dtype}")
        self.params = [p for p in params if p.requires_grad]
        self.bucket_bytes = bucket_bytes
        self.overlap = overlap
        self.grad_dtype = grad_dtype
        self._low = {}            # id(fp32 bucket) -> its bf16 staging copy
        self.segmenter = None     # SegmentedStepGraph while it captures (cuts instead of reduces)
        self.flat = []            # chunk buckets: (flat tensor, lo_layer, hi_layer)
        self.pending = []         # async work handles of this step
        self.launched = set()
        self.routed = set()       # Conformer layers whose grouped gradients all landed in the buckets
        self._no_sync = False
        self.conformer = None
        # HIP-graph steps: (captured gradient tensor, bucket view) of grouped gradients that were NOT routed into
        # their bucket at capture -- every replay rewrites the captured tensor, so allreduce() copies it in again
        # (a one-time copy + re-pointed .grad would reduce the first replay's values forever: ADVICE r3)
        self.graph_mode = False
        self._replay_src = {}
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
        """All-reduce (average) the fp32 bucket t; returns a waitable handle or None (already done)."""
        if self.grad_dtype == torch.bfloat16:
            low = self._low.get(id(t))
            if low is None or low.numel() != t.numel():
                low = torch.empty(t.numel(), device=t.device, dtype=torch.bfloat16)
                self._low[id(t)] = low
            _cast_into(t, low)
            w = self._reduce_raw(low, async_op)
            if w is None:
                _cast_into(low, t)
                return None
            return _CastBack(w, low, t)
        return self._reduce_raw(t, async_op)

    def _reduce_raw(self, t, async_op):
        op = _avg_op()
        if op is not None:
            return dist.all_reduce(t, op=op, async_op=async_op)
        w = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)
        if async_op:
            w.wait()
        t.mul_(1.0 / dist.get_world_size())
        return None

    def final_chunks(self, layer_index):
        """Chunks whose all-reduce may start once the grouped launch flushed at `layer_index` (see
        _on_flushed), not yet launched."""
        return [i for i, (flat, lo, hi) in enumerate(self.flat)
                if i not in self.launched and lo >= layer_index and all(li in self.routed for li in range(lo, hi))]

    def launch_chunk(self, i):
        """Issue chunk i's bucket all-reduce now (async; allreduce() waits for it)."""
        if i in self.launched:
            return
        self.launched.add(i)
        if self._world() == 1:
            return
        w = self._reduce(self.flat[i][0], True)
        if w is not None:
            self.pending.append(w)

    def _on_flushed(self, layer_index):
        """Called by the Conformer right after it flushed the grouped launch at `layer_index`: every chunk
        whose layers are all >= layer_index is final -> issue its all-reduce now (async).  Only chunks whose
        every grouped weight/bias gradient was WRITTEN into its bucket view by this backward's grouped launch
        (on_routed) qualify: a layer that accumulated into an existing .grad, or skipped the grouped launch
        (gradient hooks, unsupported operand shapes), finishes its gradients through AccumulateGrad AFTER
        this call, so its chunk waits for allreduce().  Nothing launches under no_sync()."""
        if self._no_sync:
            return
        if self.segmenter is not None:           # capturing a segmented step graph: cut, reduce at replay
            self.segmenter.cut(self.final_chunks(layer_index))
            return
        if self._world() == 1:
            return
        for i in self.final_chunks(layer_index):
            self.launch_chunk(i)

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
            if copy:
                src = self._replay_src.get(v.data_ptr())
                if src is not None:                 # graph replay rewrote the captured (un-routed) gradient
                    v.copy_(src.reshape(v.shape))
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                if copy:
                    v.copy_(p.grad.reshape(v.shape))
                    if self.graph_mode:
                        self._replay_src[v.data_ptr()] = p.grad
                p.grad = v.view(p.shape)

    def mark_graph(self):
        """The step's backward is now a captured HIP graph (replayed, not re-run): gradients the capture left
        outside their bucket views are copied in on every allreduce(), not only the first."""
        self.graph_mode = True
        self._replay_src = {}

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


def _cast_into(src, dst):
    if src.is_cuda:
        from . import ops
        ops.cast_into(src, dst)
    else:
        dst.copy_(src)


class _CastBack:
    """Handle of an async bf16 bucket reduce: wait() orders the stream after the collective, then casts the
    reduced bf16 copy back into the fp32 bucket."""

    def __init__(self, work, low, dst):
        self.work, self.low, self.dst = work, low, dst

    def wait(self):
        self.work.wait()
        _cast_into(self.low, self.dst)


class SegmentedStepGraph:
    """A training step's forward + backward captured as a CHAIN of HIP graphs cut where the Conformer flushes
    a gradient chunk (GradAllReducer(overlap=True) flush points, in backward order), all in ONE private memory
    pool and replayed in capture order.  After replaying segment i, the chunks that became final in it are
    all-reduced (async, RCCL's stream) while segment i+1's backward runs on the compute stream -- the
    data-parallel overlap of the eager path, with graph launch costs.  The collectives are launched from the
    host between replays, never captured.

    Usage (after one eager warm-up step, so allocator / staging tables exist):
        seg = SegmentedStepGraph(reducer); out = seg.capture(step_fn)   # step_fn: forward + backward
        loop: seg.replay(); reducer.allreduce(); optimizer.step()"""

    def __init__(self, reducer):
        if not reducer.overlap:
            raise ValueError("SegmentedStepGraph needs GradAllReducer(overlap=True) (its flush points)")
        self.reducer = reducer
        self.graphs = []          # [(CUDAGraph, [chunk indices final after it])]
        self._g = None
        self._pool = None

    def cut(self, chunks):
        """Called (through the reducer) at a flush point inside the captured backward."""
        self._g.capture_end()
        self.graphs.append((self._g, list(chunks)))
        self._g = torch.cuda.CUDAGraph()
        self._g.capture_begin(pool=self._pool, capture_error_mode="relaxed")

    def capture(self, fn):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        self._pool = torch.cuda.graph_pool_handle()
        self.graphs = []
        red = self.reducer
        red.routed = set()
        with torch.cuda.stream(s):
            # relaxed capture mode: the cuts run on autograd's device thread, not the thread that began the
            # capture (thread-local / global capture sequences must end on the thread that started them)
            self._g = torch.cuda.CUDAGraph()
            self._g.capture_begin(pool=self._pool, capture_error_mode="relaxed")
            red.segmenter = self
            try:
                out = fn()
            except BaseException:
                # end the in-flight capture so the stream leaves capture mode and the original error surfaces
                # (not a confusing capture error from the next HIP call); the partial graphs are discarded
                try:
                    self._g.capture_end()
                except Exception:
                    pass
                self._g = None
                self.graphs = []
                raise
            finally:
                red.segmenter = None
            self._g.capture_end()
            self.graphs.append((self._g, []))
            self._g = None
        torch.cuda.current_stream().wait_stream(s)
        red.launched = set()
        red.mark_graph()
        return out

    def replay(self):
        red = self.reducer
        for g, chunks in self.graphs:
            g.replay()
            for i in chunks:
                red.launch_chunk(i)

    def __len__(self):
        return len(self.graphs)


def global_batch_slice(global_batch, rank, world):
    """Contiguous slice [lo, hi) of the global utterance batch owned by `rank`."""
    per = global_batch // world
    return rank * per, (rank + 1) * per
