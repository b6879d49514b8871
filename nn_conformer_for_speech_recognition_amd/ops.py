"""Thin Python wrappers over the C ABI (include/cfm.h).  Tensors in, tensors out; every call is
stream-ordered on torch's current HIP stream and allocates only through torch's caching
allocator (so whole steps can be captured into a HIP graph)."""
from __future__ import annotations

import os

import torch

from . import _lib as L
from ._lib import ACT_NONE, ACT_SILU, BF16, F32  # noqa: F401


def _gemm_desc(**kw):
    d = L.GemmDesc()
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def gemm(A, B, C, M, N, K, *, a_kmajor=True, b_kmajor=True, lda=None, ldb=None, ldc=None, alpha=1.0,
         bias=None, act=ACT_NONE, act_grad=False, pre=None, drop_p=0.0, seed=0, offset=0, out_scale=1.0,
         residual=None, ldr=None, split_k=1, batch=1, stride_a=0, stride_b=0, stride_c=0, workspace=None,
         a_colsum=None, rowdot=None, alpha_a=None, alpha_b=None, allow_overlap=False, mx_a=None, mx_b=None,
         mx_out=None):
    """C = epilogue(alpha * A·Bᵀ) — see cfm_gemm_desc in include/cfm.h.  fp8 (e4m3fn) A and B: alpha_a /
    alpha_b are their device dequantisation scalars (quant_fp8), or mx_a / mx_b their e8m0 block scales
    (quant_mx); mx_out = (y8, s8): the MX copy of a bf16 C written by the same epilogue (fp8 FFN-up)."""
    if A.dtype != B.dtype:
        raise L.CfmError(f"gemm operands differ in dtype: {A.dtype} vs {B.dtype}")
    d = _gemm_desc(
        M=M, N=N, K=K, batch=batch, dtype_ab=L.dt(A),
        A=L.ptr(A), lda=lda if lda is not None else (K if a_kmajor else M), stride_a=stride_a, a_kmajor=int(a_kmajor),
        B=L.ptr(B), ldb=ldb if ldb is not None else (K if b_kmajor else N), stride_b=stride_b, b_kmajor=int(b_kmajor),
        C=L.ptr(C), ldc=ldc if ldc is not None else N, stride_c=stride_c, dtype_c=L.dt(C),
        alpha=float(alpha), bias=L.ptr(bias), act=int(act), act_grad=int(bool(act_grad)),
        pre=L.ptr(pre), dtype_pre=L.dt(pre) if pre is not None else F32,
        drop_p=float(drop_p), drop_seed=int(seed) & (2**64 - 1), drop_offset=int(offset),
        out_scale=float(out_scale), residual=L.ptr(residual),
        ldr=ldr if ldr is not None else N, dtype_r=L.dt(residual) if residual is not None else F32,
        split_k=int(split_k), workspace=L.ptr(workspace), a_colsum=L.ptr(a_colsum),
        rowdot_with=L.ptr(rowdot[0]) if rowdot else None, rowdot_out=L.ptr(rowdot[1]) if rowdot else None,
        rowdot_T=int(rowdot[2]) if rowdot else 0, alpha_a_dev=L.ptr(alpha_a), alpha_b_dev=L.ptr(alpha_b),
        allow_overlap=int(bool(allow_overlap)), mx_a=L.ptr(mx_a), mx_b=L.ptr(mx_b),
        mx_out=L.ptr(mx_out[0]) if mx_out else None, mx_out_scales=L.ptr(mx_out[1]) if mx_out else None)
    if PROBE is not None:
        PROBE("gemm", (M, N, K), d, lambda: L.call("cfm_gemm", L.ctypes.byref(d), L.stream()))
    else:
        L.call("cfm_gemm", L.ctypes.byref(d), L.stream())
    return C


PROBE = None   # optional timing hook (bench.py KernelProbe): PROBE(kind, shape, desc, launch)
# grouped weight gradients on the XCD-aware plan (cfm_wgrad_group_plan); CFM_WGRAD_PLAN=0 keeps the unplanned
# launch (tiles in task order, XCD-contiguous ids) for A/B
WGRAD_PLAN = os.environ.get("CFM_WGRAD_PLAN", "1") != "0"


def linear(x, w, bias=None, out_dtype=None, act=ACT_NONE, pre=None, drop_p=0.0, seed=0, offset=0,
           out_scale=1.0, residual=None, out=None, x_scale=None, w_scale=None, x_mx=None, w_mx=None, mx_out=None):
    """y = x·wᵀ (+bias, epilogue) for x (M, K), w (N, K).  fp8 operands pass their dequantisation: per-tensor
    scalars x_scale / w_scale (quant_fp8) or MX block scales x_mx / w_mx (quant_mx); the output then defaults to
    bf16."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        od = out_dtype or (torch.bfloat16 if x.dtype == torch.float8_e4m3fn else x.dtype)
        out = torch.empty(M, N, device=x.device, dtype=od)
    return gemm(x, w, out, M, N, K, bias=bias, act=act, pre=pre, drop_p=drop_p, seed=seed, offset=offset,
                out_scale=out_scale, residual=residual, alpha_a=x_scale, alpha_b=w_scale, mx_a=x_mx, mx_b=w_mx,
                mx_out=mx_out)


def quant_fp8(x, out=None, inv_scale=None):
    """Per-tensor e4m3fn quantisation on the device: (y float8_e4m3fn of x's shape, inv_scale (1,) fp32)
    with y = e4m3(x * 2^k), k the largest with amax|x| * 2^k <= 448, and inv_scale = 2^-k (cfm_quant_fp8)."""
    if not x.is_contiguous():
        raise L.CfmError("quant_fp8: contiguous input required")
    y = out if out is not None else torch.empty(x.shape, device=x.device, dtype=torch.float8_e4m3fn)
    sc = inv_scale if inv_scale is not None else torch.empty(1, device=x.device, dtype=torch.float32)
    ws = workspace(L.size_call("cfm_quant_fp8_ws_bytes"), x.device)
    L.call("cfm_quant_fp8", L.ptr(x), L.dt(x), x.numel(), L.ptr(y), L.ptr(sc), L.ptr(ws), L.stream())
    return y, sc


def quant_mx(x, out=None, scales=None):
    """MX e4m3 quantisation on the device (cfm_quant_mx): x (rows, K), K % 32 == 0 -> (y float8_e4m3fn (rows, K),
    s uint8 (rows, K/32) e8m0 block scales): y = e4m3(x * 2^k) per 32-element block, k the largest with
    amax(block) * 2^k <= 448, s = 127 - k."""
    if x.dim() != 2 or not x.is_contiguous():
        raise L.CfmError("quant_mx: contiguous 2-D input required")
    rows, K = x.shape
    y = out if out is not None else torch.empty(rows, K, device=x.device, dtype=torch.float8_e4m3fn)
    s = scales if scales is not None else torch.empty(rows, K // 32, device=x.device, dtype=torch.uint8)
    L.call("cfm_quant_mx", L.ptr(x), L.dt(x), rows, K, K, L.ptr(y), L.ptr(s), L.stream())
    return y, s


def dequant_mx(y, s):
    """float32 view of an MX tensor: e4m3(y) * 2^(s - 127) per 32-element block (tests)."""
    out = torch.empty(y.shape, device=y.device, dtype=torch.float32)
    L.call("cfm_dequant_mx", L.ptr(y), L.ptr(s), y.numel(), L.ptr(out), L.stream())
    return out


def linear_dgrad(dy, w, out_dtype=None, pre=None, act_grad=False, drop_p=0.0, seed=0, offset=0, out=None,
                 wt=None, rowdot=None):
    """dx = dy·w for dy (M, N), w (N, K); optional silu'/dropout-mask epilogue (backward of the
    producing GEMM's epilogue).  wt: optional (K, N) row-major copy of wᵀ (CastTBatch) -- then both
    operands are read K-major, the faster GEMM path."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=out_dtype or dy.dtype)
    if wt is not None:
        if tuple(wt.shape) != (K, N) or not wt.is_contiguous() or wt.dtype != dy.dtype:
            raise L.CfmError(f"linear_dgrad: wt must be a contiguous ({K}, {N}) {dy.dtype} copy of w^T")
        return gemm(dy, wt, out, M, K, N, a_kmajor=True, b_kmajor=True, lda=N, ldb=N, act_grad=act_grad, pre=pre,
                    drop_p=drop_p, seed=seed, offset=offset, rowdot=rowdot)
    return gemm(dy, w, out, M, K, N, a_kmajor=True, b_kmajor=False, lda=N, ldb=K, act_grad=act_grad, pre=pre,
                drop_p=drop_p, seed=seed, offset=offset)


# fusions that can be switched off for same-box A/B timing: CFM_DISABLE="rowdot,lndrop,wgbias"
DISABLED = frozenset(x for x in os.environ.get("CFM_DISABLE", "").split(",") if x)
ENABLED = frozenset(x for x in os.environ.get("CFM_ENABLE", "").split(",") if x)   # opt-in variants (A/B)

# target workgroup count (in 128x128-tile units) of the split-K weight-gradient GEMMs
_WGRAD_WGS = int(os.environ.get("CFM_WGRAD_WGS", "512"))


def linear_wgrad(dy, x, out=None, split_k=None, bias_out=None):
    """dW = dyᵀ·x for dy (M, N), x (M, K) → (N, K) fp32 (token dim reduced; both operands stay
    token-major in HBM and are transposed by ds_read_b64_tr_b16 on the way into the MFMAs).
    bias_out: optional (N,) fp32 <- Σ_rows dy (the bias gradient), taken from the same GEMM's staged
    dy tiles and split-K reduction when the LDS-DMA path runs it, else by cfm_colsum."""
    M, N = dy.shape
    K = x.shape[1]
    if split_k is None:
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        split_k = max(1, min(16, _WGRAD_WGS // max(tiles, 1), M // 1024))
    if out is None:
        out = torch.empty(N, K, device=dy.device, dtype=torch.float32)
    ws = None
    fused = False
    if split_k > 1:
        if K % 4 == 0:       # deterministic slab reduction (no atomics, no zero-fill)
            fused = (bias_out is not None and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
                     and N % 8 == 0 and K % 8 == 0 and dy.is_contiguous() and x.is_contiguous())
            ws = torch.empty(split_k * N * K + (split_k * N if fused else 0), device=dy.device, dtype=torch.float32)
        else:
            out.zero_()
    gemm(dy, x, out, N, K, M, a_kmajor=False, b_kmajor=False, lda=N, ldb=K, split_k=split_k, workspace=ws,
         a_colsum=bias_out if fused else None)
    if bias_out is not None and not fused:
        colsum(dy, out=bias_out)
    return out


class _ProbeDesc:
    """Launch descriptor stand-in for PROBE hooks of non-GEMM launches (only .probe is read)."""
    probe = None


class WgradGroup:
    """Deferred weight gradients: add(dy, x) returns (dW, db) tensors that flush() fills with ONE grouped
    launch (cfm_wgrad_group) -- dW = dyᵀ·x, db = Σ_rows dy, bf16 operands sharing the token count M.
    The returned tensors must not be read before flush() (they are views, so autograd's AccumulateGrad
    adopts them without a copy).  Tables are cached by operand pointers (fixed under graph replay)."""

    POOL_BYTES = 8 << 20     # pinned staging for the task tables (allocated at the first, eager, flush)
    CAPTURE_POOL_BYTES = 2 << 20

    def __init__(self):
        self.tasks = []
        self._cache = {}
        self._pool = None        # eager tables: ring (a slice is only re-read by its own, finished, copy)
        self._cpool = None       # tables staged inside a graph capture: bump-allocated, never reused
        self._off = 0
        self._coff = 0
        self._armed = False
        self._stream = None

    def _stage(self, host):
        """Copy a host table to the device through a slice of a persistent pinned pool: legal inside a
        HIP-graph capture (pageable copies and pinned allocations are not).  A captured copy node re-reads
        its host slice on every replay, so slices staged under capture come from a separate bump-only pool
        that is never recycled (eager flushes wrapping the ring cannot overwrite them)."""
        n = host.nbytes
        capturing = torch.cuda.is_current_stream_capturing()
        if self._pool is None:
            if capturing:
                raise L.CfmError("WgradGroup: first flush inside a graph capture; run one eager step first")
            self._pool = torch.empty(max(self.POOL_BYTES, n), dtype=torch.uint8).pin_memory()
            self._cpool = torch.empty(self.CAPTURE_POOL_BYTES, dtype=torch.uint8).pin_memory()
        if capturing:
            if self._coff + n > self._cpool.numel():
                raise L.CfmError("WgradGroup: capture staging pool exhausted (too many distinct captured flushes)")
            dst = self._cpool[self._coff:self._coff + n]
            self._coff += (n + 255) // 256 * 256
        else:
            if self._off + n > self._pool.numel():
                self._off = 0
            dst = self._pool[self._off:self._off + n]
            self._off += (n + 255) // 256 * 256
        dst.numpy()[:] = host
        return dst.to(self.tasks[0][0].device, non_blocking=True)

    def __len__(self):
        return len(self.tasks)

    def arm_final_flush(self):
        """Safety net for a backward in which the flushing layer (layer 0) never runs (pruned node): an
        end-of-backward engine callback flushes whatever is still queued, on the stream the tasks were
        queued from, so no deferred gradient outlives its backward pass unfilled."""
        if self._armed:
            return
        self._armed = True

        def _final():
            self._armed = False
            if self.tasks:
                with torch.cuda.stream(self._stream):
                    self.flush()
        torch.autograd.Variable._execution_engine.queue_callback(_final)

    def add(self, dy, x, dest=None):
        """dest: optional (dW (N, K), db (N,)) fp32 destinations (e.g. views of a data-parallel gradient
        bucket); fresh views of them are returned, so autograd adopts them as .grad without a copy."""
        M, N = dy.shape
        K = x.shape[1]
        if dest is not None:
            dw, db = dest
            if tuple(dw.shape) != (N, K) or tuple(db.shape) != (N,) or not dw.is_contiguous():
                raise L.CfmError("WgradGroup.add: destination shapes do not match the GEMM")
        else:
            dw = torch.empty(N, K, device=dy.device, dtype=torch.float32)
            db = torch.empty(N, device=dy.device, dtype=torch.float32)
        self.tasks.append((dy, x, dw, db))
        self._stream = torch.cuda.current_stream(dy.device)
        return dw.view(N, K), db.view(N)

    def _plan(self, dev, lib):
        """cfm_wgrad_group_plan over the queued tasks: (schedule words (grid,), per-task split factors)."""
        import numpy as np
        n = len(self.tasks)
        tiles = np.array([lib.cfm_wgrad_group_tiles(t[0].shape[1], t[1].shape[1]) for t in self.tasks], dtype=np.int64)
        nxcd = 8                                       # MI355X: 8 XCDs (placement is a speed hint only)
        cus = max(1, torch.cuda.get_device_properties(dev).multi_processor_count // nxcd)
        cap = int(tiles.sum()) * 16 + 64 * nxcd
        sched = np.empty(cap, dtype=np.uint32)
        split = np.ones(n, dtype=np.int32)
        grid = lib.cfm_wgrad_group_plan(tiles.ctypes.data, n, nxcd, cus, sched.ctypes.data, cap, split.ctypes.data)
        if grid <= 0:
            raise L.CfmError("cfm_wgrad_group_plan failed: " + lib.cfm_get_last_error().decode(errors="replace"))
        return sched[:grid].copy(), split

    def flush(self):
        if not self.tasks:
            return
        import numpy as np
        dev = self.tasks[0][0].device
        # (the tile width of the launch variant is part of the table: cfm_wgrad_group_tiles(256, 256) is 1 or 2)
        key = tuple((t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), t[0].shape[0],
                     t[0].shape[1], t[1].shape[1]) for t in self.tasks) + (L.load().cfm_wgrad_group_tiles(256, 256),
                                                                           WGRAD_PLAN)
        hit = self._cache.get(key)
        if hit is None:
            lib = L.load()
            tb = L.size_call("cfm_wgrad_group_task_bytes")
            host = np.zeros(tb * len(self.tasks), dtype=np.uint8)
            captured = torch.cuda.is_current_stream_capturing()
            if WGRAD_PLAN:
                sched, split = self._plan(dev, lib)
                shapes = [(t[0].shape[1], t[1].shape[1]) for t in self.tasks]
                wsf = [lib.cfm_wgrad_group_ws_floats(N, K, int(s)) for (N, K), s in zip(shapes, split)]
                ws = torch.empty(max(1, sum(wsf)), dtype=torch.float32, device=dev) if sum(wsf) else None
                off = red0 = 0
                for i, (dy, x, dw, db) in enumerate(self.tasks):
                    M, N = dy.shape
                    K = x.shape[1]
                    wp = ws.data_ptr() + 4 * off if wsf[i] else None
                    L.call("cfm_wgrad_group_fill_split", host.ctypes.data, i, L.ptr(dy), L.ptr(x), L.ptr(dw),
                           L.ptr(db), M, N, K, int(split[i]), wp, red0)
                    off += wsf[i]
                    red0 += lib.cfm_wgrad_group_red_blocks(N, K, int(split[i]))
                table = self._stage(host)
                hit = (captured, table, len(sched), self._stage(sched.view(np.uint8)), red0, ws)
            else:
                tile0 = 0
                for i, (dy, x, dw, db) in enumerate(self.tasks):
                    M, N = dy.shape
                    K = x.shape[1]
                    L.call("cfm_wgrad_group_fill", host.ctypes.data, i, L.ptr(dy), L.ptr(x), L.ptr(dw), L.ptr(db), M,
                           N, K, tile0)
                    tile0 += lib.cfm_wgrad_group_tiles(N, K)
                table = self._stage(host)
                hit = (captured, table, tile0)
            if len(self._cache) > 8:
                # a captured graph's kernel node holds the device table's address: keep those entries
                self._cache = {k: v for k, v in self._cache.items() if v[0]}
            self._cache[key] = hit
        desc = _ProbeDesc()
        n = len(self.tasks)

        def launch():
            if len(hit) > 3:
                L.call("cfm_wgrad_group_sched", L.ptr(hit[1]), n, L.ptr(hit[3]), hit[2], hit[4], desc.probe,
                       L.stream())
                return
            L.call("cfm_wgrad_group_probed", L.ptr(hit[1]), n, hit[2], desc.probe, L.stream())
        if PROBE is not None:
            PROBE("wgroup", (n, hit[2]), desc, launch)
        else:
            launch()
        self.tasks = []


class ReduceGroup(WgradGroup):
    """Deferred small column reductions of a backward pass (LayerNorm dgamma|dbeta partial rows, depthwise-conv
    weight/bias partials) flushed as ONE cfm_colreduce_group launch -- instead of ~85 tiny side-stream
    launches per Conformer-L step.  Outputs must not be read before flush() (same contract as WgradGroup;
    the staging pools and the capture rules are WgradGroup's)."""

    def add_sum(self, part, nparts, N, ldp, out):
        """out[n] = sum_p part[p*ldp + n]; the caller hands autograd fresh views of out (see add_dwconv)."""
        self.tasks.append((part, out, None, int(nparts), int(N), int(ldp), 0, 0, 0))
        self._stream = torch.cuda.current_stream(part.device)

    def add_dwconv(self, part, nparts, C, K, dw, db):
        """the depthwise conv's [nparts][K+1][C] partials -> dw (C, K), db (C).  Returns fresh views of
        dw / db: the task keeps the tensors themselves, and autograd adopts a gradient without a copy only
        when nothing else references it (a copy taken before flush() would hold garbage)."""
        N = C * (K + 1)
        self.tasks.append((part, dw, db, int(nparts), N, N, 1, int(C), int(K)))
        self._stream = torch.cuda.current_stream(part.device)
        return dw.view(C, K), db.view(C)

    def flush(self):
        if not self.tasks:
            return
        import numpy as np
        key = tuple((t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr() if t[2] is not None else 0) + t[3:]
                    for t in self.tasks)
        hit = self._cache.get(key)
        if hit is None:
            lib = L.load()
            tb = L.size_call("cfm_colreduce_group_task_bytes")
            host = np.zeros(tb * len(self.tasks), dtype=np.uint8)
            blk0 = 0
            for i, (part, out, out2, nparts, N, ldp, mode, C, K) in enumerate(self.tasks):
                L.call("cfm_colreduce_group_fill", host.ctypes.data, i, L.ptr(part), nparts, N, ldp, L.ptr(out),
                       L.ptr(out2), mode, C, K, blk0)
                blk0 += lib.cfm_colreduce_group_blocks(N)
            captured = torch.cuda.is_current_stream_capturing()
            table = self._stage(host)
            hit = (captured, table, blk0)
            if len(self._cache) > 8:
                self._cache = {k: v for k, v in self._cache.items() if v[0]}
            self._cache[key] = hit
        L.call("cfm_colreduce_group", L.ptr(hit[1]), len(self.tasks), hit[2], L.stream())
        self.tasks = []


def wgrad_group_ok(dy, x):
    """Operands the grouped weight-gradient launch takes (else linear_wgrad per GEMM)."""
    return (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.is_contiguous() and x.is_contiguous()
            and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0
            and dy.numel() * 2 < 2 ** 31 and x.numel() * 2 < 2 ** 31)


_ws_cache = {}


def workspace(nbytes, device, tag="ws"):
    """Workspace from torch's allocator (a fresh tensor: safe under graph capture / streams)."""
    n = (int(nbytes) + 3) // 4
    return torch.empty(max(n, 1), device=device, dtype=torch.float32)


def colsum(x, out=None, accumulate=False):
    M, N = x.shape
    if out is None:
        out = torch.empty(N, device=x.device, dtype=torch.float32)
    ws = workspace(4 * N * 256, x.device)
    L.call("cfm_colsum", L.ptr(x), L.dt(x), M, N, x.stride(0), L.ptr(out), int(accumulate), L.ptr(ws), L.stream())
    return out


def cast(x, dtype):
    y = torch.empty(x.shape, device=x.device, dtype=dtype)
    L.call("cfm_cast", L.ptr(x), L.dt(x), L.ptr(y), L.dt(y), x.numel(), L.stream())
    return y


_CAST_BLK = 2048


class CastBatch:
    """One launch that casts a fixed list of tensors into fixed destination tensors (cfm_cast_batch).
    The device task table is built once; call refresh() to re-run the casts (e.g. the bf16 shadow
    of every weight matrix, once per step)."""

    def __init__(self, srcs, dsts):
        import numpy as np
        if not srcs or len(srcs) != len(dsts):
            raise L.CfmError("CastBatch: need matching non-empty source / destination lists")
        dtx, dty = {L.dt(t) for t in srcs}, {L.dt(t) for t in dsts}
        if len(dtx) != 1 or len(dty) != 1:
            raise L.CfmError("CastBatch: one source dtype and one destination dtype per batch")
        self.dtx, self.dty = dtx.pop(), dty.pop()
        rec = np.zeros((len(srcs), 4), dtype=np.int64)
        blk = 0
        for i, (s, d) in enumerate(zip(srcs, dsts)):
            if s.numel() != d.numel() or not s.is_contiguous() or not d.is_contiguous():
                raise L.CfmError("CastBatch: contiguous tensors of equal size required")
            rec[i] = (L.ptr(s), L.ptr(d), s.numel(), blk)
            blk += (s.numel() + _CAST_BLK - 1) // _CAST_BLK
        self.nblocks = blk
        self.table = torch.from_numpy(rec.view(np.uint8).reshape(-1).copy()).to(srcs[0].device)
        self.n = len(srcs)
        self._keep = (list(srcs), list(dsts))

    def refresh(self):
        L.call("cfm_cast_batch", L.ptr(self.table), self.n, self.nblocks, self.dtx, self.dty, L.stream())


class CastTBatch:
    """One launch that writes transposed compute-dtype copies dst = srcᵀ of a fixed list of 2-D
    fp32 tensors (cfm_cast_transpose_batch): the K-major weight copies of the data-gradient GEMMs;
    with dsts_n also the plain copies dsts_n = src from the same read (the per-step bf16 shadow)."""

    def __init__(self, srcs, dsts, dsts_n=None):
        import numpy as np
        if not srcs or len(srcs) != len(dsts):
            raise L.CfmError("CastTBatch: need matching non-empty source / destination lists")
        dtx, dty = {L.dt(t) for t in srcs}, {L.dt(t) for t in dsts}
        if len(dtx) != 1 or len(dty) != 1:
            raise L.CfmError("CastTBatch: one source dtype and one destination dtype per batch")
        self.dtx, self.dty = dtx.pop(), dty.pop()
        if self.dtx != L.F32:
            raise L.CfmError("CastTBatch: fp32 sources only")
        if dsts_n is not None and (len(dsts_n) != len(srcs) or {L.dt(t) for t in dsts_n} != {self.dty}):
            raise L.CfmError("CastTBatch: dsts_n must match srcs in count and dsts in dtype")
        rec = np.zeros((len(srcs), 6), dtype=np.int64)
        blk = 0
        for i, (s, d) in enumerate(zip(srcs, dsts)):
            if s.dim() != 2 or tuple(d.shape) != (s.shape[1], s.shape[0]) or not s.is_contiguous() \
                    or not d.is_contiguous():
                raise L.CfmError("CastTBatch: contiguous 2-D source and its transposed-shape destination required")
            pn = 0
            if dsts_n is not None:
                dn = dsts_n[i]
                if dn.numel() != s.numel() or not dn.is_contiguous():
                    raise L.CfmError("CastTBatch: contiguous plain destination of the source's size required")
                pn = L.ptr(dn)
            rec[i] = (L.ptr(s), L.ptr(d), pn, s.shape[0], s.shape[1], blk)
            blk += ((s.shape[0] + 63) // 64) * ((s.shape[1] + 63) // 64)
        self.nblocks = blk
        self.table = torch.from_numpy(rec.view(np.uint8).reshape(-1).copy()).to(srcs[0].device)
        self.n = len(srcs)
        self._keep = (list(srcs), list(dsts), list(dsts_n or []))

    def refresh(self):
        L.call("cfm_cast_transpose_batch", L.ptr(self.table), self.n, self.nblocks, self.dtx, self.dty, L.stream())


class Quant8Batch:
    """Per-step e4m3 copies of a fixed list of tensors in TWO launches (cfm_quant_fp8_batch): the same current
    scaling, scales and bytes as quant_fp8 per tensor.  outs[i] = (y float8_e4m3fn of srcs[i]'s shape,
    inv_scale (1,) fp32), persistent across refresh() calls (graph-capturable: the table is built once)."""

    def __init__(self, srcs):
        import numpy as np
        if not srcs:
            raise L.CfmError("Quant8Batch: empty list")
        dts = {L.dt(t) for t in srcs}
        if len(dts) != 1 or dts & {L.F32, L.BF16} != dts:
            raise L.CfmError("Quant8Batch: one fp32 or bf16 source dtype per batch")
        self.dtx = dts.pop()
        dev = srcs[0].device
        self.outs = []
        rec = np.zeros((len(srcs), 5), dtype=np.int64)
        blk = 0
        for i, x in enumerate(srcs):
            if not x.is_contiguous() or L.ptr(x) % 16:
                raise L.CfmError("Quant8Batch: contiguous 16-B aligned sources required")
            y = torch.empty(x.shape, device=dev, dtype=torch.float8_e4m3fn)
            sc = torch.empty(1, device=dev, dtype=torch.float32)
            self.outs.append((y, sc))
            rec[i] = (L.ptr(x), L.ptr(y), L.ptr(sc), x.numel(), blk)
            blk += L.load().cfm_quant_fp8_batch_blocks(x.numel())
        self.nblocks = blk
        self.table = torch.from_numpy(rec.view(np.uint8).reshape(-1).copy()).to(dev)
        self.part = torch.empty(blk, device=dev, dtype=torch.float32)
        self._keep = list(srcs)

    def refresh(self):
        L.call("cfm_quant_fp8_batch", L.ptr(self.table), len(self.outs), self.nblocks, self.dtx, L.ptr(self.part),
               L.stream())
        return self.outs


class QuantMXBatch:
    """Per-step MX e4m3 copies of a fixed list of 2-D tensors (rows, K) in ONE launch (cfm_quant_mx_batch): the
    same bytes and block scales as quant_mx per tensor.  outs[i] = (y float8_e4m3fn (rows, K), s uint8 (rows, K/32)),
    persistent across refresh() calls (graph-capturable: the table is built once)."""

    def __init__(self, srcs):
        import numpy as np
        if not srcs:
            raise L.CfmError("QuantMXBatch: empty list")
        dts = {L.dt(t) for t in srcs}
        if len(dts) != 1 or dts & {L.F32, L.BF16} != dts:
            raise L.CfmError("QuantMXBatch: one fp32 or bf16 source dtype per batch")
        self.dtx = dts.pop()
        dev = srcs[0].device
        self.outs = []
        rec = np.zeros((len(srcs), 6), dtype=np.int64)   # cfm_mx_task: x, y, s, rows, (K | pad), blk0
        blk = 0
        for i, x in enumerate(srcs):
            if x.dim() != 2 or not x.is_contiguous() or L.ptr(x) % 16 or x.shape[1] % 32:
                raise L.CfmError("QuantMXBatch: contiguous 16-B aligned (rows, K) sources, K % 32 == 0")
            rows, K = x.shape
            y = torch.empty(rows, K, device=dev, dtype=torch.float8_e4m3fn)
            s = torch.empty(rows, K // 32, device=dev, dtype=torch.uint8)
            self.outs.append((y, s))
            rec[i] = (L.ptr(x), L.ptr(y), L.ptr(s), rows, K, blk)
            blk += L.load().cfm_quant_mx_batch_blocks(rows, K)
        self.nblocks = blk
        self.table = torch.from_numpy(rec.view(np.uint8).reshape(-1).copy()).to(dev)
        self._keep = list(srcs)

    def refresh(self):
        L.call("cfm_quant_mx_batch", L.ptr(self.table), len(self.outs), self.nblocks, self.dtx, L.stream())
        return self.outs


def cast_into(x, y):
    L.call("cfm_cast", L.ptr(x), L.dt(x), L.ptr(y), L.dt(y), x.numel(), L.stream())
    return y


def layernorm_fwd(x, gamma, beta, eps=1e-5, out_dtype=None):
    M, D = x.shape
    y = torch.empty(M, D, device=x.device, dtype=out_dtype or x.dtype)
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    L.call("cfm_layernorm_fwd", L.ptr(x), L.dt(x), L.ptr(gamma), L.ptr(beta), L.ptr(y), L.dt(y), L.ptr(mean),
           L.ptr(rstd), M, D, float(eps), L.stream())
    return y, mean, rstd


def layernorm_fwd_mx(x, gamma, beta, eps=1e-5):
    """layernorm_fwd with a bf16 y AND its MX e4m3 copy from the same kernel: (y, (y8, s8), mean, rstd), y8 / s8
    exactly quant_mx(y) (cfm_layernorm_fwd_mx)."""
    M, D = x.shape
    y = torch.empty(M, D, device=x.device, dtype=torch.bfloat16)
    y8 = torch.empty(M, D, device=x.device, dtype=torch.float8_e4m3fn)
    s8 = torch.empty(M, D // 32, device=x.device, dtype=torch.uint8)
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    L.call("cfm_layernorm_fwd_mx_ex", L.ptr(x), L.dt(x), L.ptr(gamma), L.ptr(beta), L.ptr(y), L.ptr(y8), L.ptr(s8),
           L.ptr(mean), L.ptr(rstd), M, D, float(eps), L.stream())
    return y, (y8, s8), mean, rstd


def layernorm_fwd_res(x, delta, gamma, beta, eps=1e-5, out_dtype=None, mx=False):
    """x' = x + delta (fp32, a new tensor) and LayerNorm(x') from one kernel (cfm_layernorm_fwd_res): the residual add
    of the module before the LayerNorm, whose GEMM wrote delta (bf16) without the residual.
    -> (x', y, mean, rstd), or with mx=True (bf16 y and its MX e4m3 copy) (x', y, (y8, s8), mean, rstd)."""
    M, D = x.shape
    if x.dtype != torch.float32 or delta.shape != x.shape:
        raise L.CfmError("layernorm_fwd_res: fp32 x and a delta of x's shape")
    x = x.contiguous()
    delta = delta.contiguous()
    xo = torch.empty_like(x)
    yd = torch.bfloat16 if mx else (out_dtype or x.dtype)
    y = torch.empty(M, D, device=x.device, dtype=yd)
    y8 = torch.empty(M, D, device=x.device, dtype=torch.float8_e4m3fn) if mx else None
    s8 = torch.empty(M, D // 32, device=x.device, dtype=torch.uint8) if mx else None
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    L.call("cfm_layernorm_fwd_res", L.ptr(x), L.ptr(delta), L.dt(delta), L.ptr(xo), L.ptr(gamma), L.ptr(beta),
           L.ptr(y), L.dt(y), L.ptr(y8) if mx else None, L.ptr(s8) if mx else None, L.ptr(mean), L.ptr(rstd), M, D,
           float(eps), L.stream())
    if mx:
        return xo, y, (y8, s8), mean, rstd
    return xo, y, mean, rstd


def layernorm_bwd(dy, x, gamma, mean, rstd, dres=None, dx_dtype=torch.float32, side=None, drop=None):
    """dx (+ dres) and (dgamma, dbeta).  side: optional object with run(fn, *keep) (conformer._Side):
    the dgamma|dbeta partial-row reduction is then launched there, off the data-gradient chain.
    drop: optional (scale, p, seed, dtype) -> also returns g2 = scale_dropout(dx, scale, p, seed) in
    `dtype`, written by the same kernel (4 return values then)."""
    M, D = x.shape
    dx = torch.empty(M, D, device=x.device, dtype=dx_dtype)
    gb = torch.empty(2, D, device=x.device, dtype=torch.float32)   # adjacent: one reduction pass
    dgamma, dbeta = gb[0], gb[1]
    ws = workspace(L.size_call("cfm_layernorm_ws_bytes", M, D), x.device)
    defer = side is not None
    g2 = None
    if drop is not None and drop[3] == torch.bfloat16:
        scale, p, seed = float(drop[0]), float(drop[1]), int(drop[2])
        g2 = torch.empty(M, D, device=x.device, dtype=torch.bfloat16)
        L.call("cfm_layernorm_bwd_drop", L.ptr(dy), L.dt(dy), L.ptr(x), L.dt(x), L.ptr(gamma), L.ptr(mean),
               L.ptr(rstd), L.ptr(dres), L.dt(dres), L.ptr(dx), L.dt(dx), None if defer else L.ptr(dgamma),
               None if defer else L.ptr(dbeta), L.ptr(ws), M, D, L.ptr(g2), scale, p, seed, L.stream())
    else:
        L.call("cfm_layernorm_bwd", L.ptr(dy), L.dt(dy), L.ptr(x), L.dt(x), L.ptr(gamma), L.ptr(mean), L.ptr(rstd),
               L.ptr(dres), L.dt(dres), L.ptr(dx), L.dt(dx), None if defer else L.ptr(dgamma),
               None if defer else L.ptr(dbeta), L.ptr(ws), M, D, L.stream())
        if drop is not None:
            g2 = scale_dropout(dx, drop[0], drop[1], drop[2], 0, out_dtype=drop[3])
    if defer:
        nb = (L.size_call("cfm_layernorm_ws_bytes", M, D) // 4 - 2 * D) // (2 * D)
        if getattr(side, "rgroup", None) is not None:      # one grouped reduction at the end of backward
            side.rgroup.add_sum(ws, nb, 2 * D, 2 * D, gb)
        else:
            side.run(lambda: L.call("cfm_colreduce", L.ptr(ws), nb, 2 * D, 2 * D, L.ptr(gb), 0, L.stream()), ws, gb)
    if drop is not None:
        return dx, dgamma, dbeta, g2
    return dx, dgamma, dbeta


def scale_dropout(x, scale=1.0, drop_p=0.0, seed=0, offset=0, out_dtype=None):
    y = torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    L.call("cfm_scale_dropout", L.ptr(x), L.dt(x), L.ptr(y), L.dt(y), x.numel(), float(scale), float(drop_p),
           int(seed) & (2**64 - 1), int(offset), L.stream())
    return y


def specaug_apply(x, params_dev, intended=False, mask_value=0.0):
    """x (B, F, T) fp32 on GPU; params_dev int32 on GPU (see include/cfm.h)."""
    B, F, T = x.shape
    y = torch.empty_like(x)
    L.call("cfm_specaug_apply", L.ptr(x), L.ptr(y), B, F, T, L.ptr(params_dev), params_dev.numel(),
           int(bool(intended)), float(mask_value), L.stream())
    return y


def silu_bwd(dy, pre, out_dtype=None):
    dx = torch.empty(dy.shape, device=dy.device, dtype=out_dtype or dy.dtype)
    L.call("cfm_silu_bwd", L.ptr(dy), L.dt(dy), L.ptr(pre), L.dt(pre), L.ptr(dx), L.dt(dx), dy.numel(), L.stream())
    return dx


def bn_fwd(y, gamma, beta, running_mean, running_var, momentum, eps, training, act=0, out_dtype=torch.float32):
    M, C = y.shape
    mean = torch.empty(C, device=y.device, dtype=torch.float32)
    invstd = torch.empty(C, device=y.device, dtype=torch.float32)
    z = torch.empty(M, C, device=y.device, dtype=out_dtype)
    ws = workspace(L.size_call("cfm_bn_ws_bytes", C), y.device)
    L.call("cfm_bn_fwd", L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(running_mean), L.ptr(running_var),
           float(momentum), float(eps), int(bool(training)), L.ptr(mean), L.ptr(invstd), L.ptr(z), L.dt(z), M, C,
           int(act), L.ptr(ws), L.stream())
    return z, mean, invstd


def bn_bwd(dz, y, gamma, beta, mean, invstd, training, act=0):
    M, C = y.shape
    dy = torch.empty(M, C, device=y.device, dtype=torch.float32)
    dgamma = torch.empty(C, device=y.device, dtype=torch.float32)
    dbeta = torch.empty(C, device=y.device, dtype=torch.float32)
    ws = workspace(L.size_call("cfm_bn_ws_bytes", C), y.device)
    L.call("cfm_bn_bwd", L.ptr(dz), L.dt(dz), L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(mean), L.ptr(invstd),
           int(bool(training)), int(act), L.ptr(dy), L.ptr(dgamma), L.ptr(dbeta), M, C, L.ptr(ws), L.stream())
    return dy, dgamma, dbeta


# ----------------------------------------------------------------------------- convolution module
def convmod_ws(B, T, C, K, device):
    return workspace(L.size_call("cfm_convmod_ws_bytes", B, T, C, K), device)


def glu_dwconv_fwd(a, w_dw, b_dw, B, T, C, K, ws):
    y = torch.empty(B * T, C, device=a.device, dtype=torch.float32)
    L.call("cfm_glu_dwconv_fwd", L.ptr(a), L.dt(a), L.ptr(w_dw), L.ptr(b_dw), L.ptr(y), B, T, C, K, L.ptr(ws),
           L.stream())
    return y


def bn_silu_fwd(y, gamma, beta, running_mean, running_var, momentum, eps, training, B, T, C, ws, out_dtype):
    mean = torch.empty(C, device=y.device, dtype=torch.float32)
    invstd = torch.empty(C, device=y.device, dtype=torch.float32)
    z = torch.empty(B * T, C, device=y.device, dtype=out_dtype)
    L.call("cfm_bn_silu_fwd", L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(running_mean), L.ptr(running_var),
           float(momentum), float(eps), int(bool(training)), L.ptr(mean), L.ptr(invstd), L.ptr(z), L.dt(z), B, T, C,
           L.ptr(ws), L.stream())
    return z, mean, invstd


def bn_silu_fwd_sync(y, gamma, beta, running_mean, running_var, momentum, eps, B, T, C, ws, out_dtype, reduce_sums,
                     world):
    """SyncBatchNorm forward (train mode): this rank's (sum, sumsq) from the dwconv partials in ws, summed
    over the replicas by reduce_sums(tensor) (an in-place all-reduce), then stats over world*B*T rows."""
    sums = torch.empty(2 * C, device=y.device, dtype=torch.float32)
    L.call("cfm_bn_silu_fwd_sums", L.ptr(ws), B, T, C, L.ptr(sums), L.stream())
    reduce_sums(sums)
    mean = torch.empty(C, device=y.device, dtype=torch.float32)
    invstd = torch.empty(C, device=y.device, dtype=torch.float32)
    z = torch.empty(B * T, C, device=y.device, dtype=out_dtype)
    L.call("cfm_bn_silu_fwd_apply", L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(running_mean), L.ptr(running_var),
           float(momentum), float(eps), L.ptr(sums), int(world) * B * T, L.ptr(mean), L.ptr(invstd), L.ptr(z), L.dt(z),
           B * T, C, L.stream())
    return z, mean, invstd


def bn_silu_bwd_sync(dz, y, gamma, beta, mean, invstd, ws, reduce_sums, world):
    """SyncBatchNorm backward: (dgamma, dbeta) stay this rank's (the parameter gradients, averaged later
    with the others); a summed copy over the replicas feeds the input gradient."""
    M, C = y.shape
    dbg = torch.empty(2, C, device=y.device, dtype=torch.float32)
    L.call("cfm_bn_silu_bwd_sums", L.ptr(dz), L.dt(dz), L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(mean),
           L.ptr(invstd), M, C, L.ptr(ws), L.ptr(dbg[0]), L.ptr(dbg[1]), L.stream())
    tot = dbg.clone()
    reduce_sums(tot)
    dy = torch.empty(M, C, device=y.device, dtype=torch.float32)
    L.call("cfm_bn_silu_bwd_apply", L.ptr(dz), L.dt(dz), L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(mean),
           L.ptr(invstd), L.ptr(tot[0]), L.ptr(tot[1]), int(world) * M, L.ptr(dy), M, C, L.stream())
    return dy, dbg[1], dbg[0]


def bn_silu_bwd(dz, y, gamma, beta, mean, invstd, training, ws):
    M, C = y.shape
    dy = torch.empty(M, C, device=y.device, dtype=torch.float32)
    dgamma = torch.empty(C, device=y.device, dtype=torch.float32)
    dbeta = torch.empty(C, device=y.device, dtype=torch.float32)
    L.call("cfm_bn_silu_bwd", L.ptr(dz), L.dt(dz), L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(mean), L.ptr(invstd),
           int(bool(training)), L.ptr(dy), L.ptr(dgamma), L.ptr(dbeta), M, C, L.ptr(ws), L.stream())
    return dy, dgamma, dbeta


# kernel sizes with a compiled depthwise variant (convmod.hip CFM_K_CASES); the BN-folded backward needs one
BN_FOLD_K = (3, 5, 7, 15, 31, 33)


def glu_dwconv_bwd(dy, a, w_dw, B, T, C, K, ws, da_dtype, side=None):
    """side: optional conformer._Side -- the depthwise weight/bias reduction then runs there."""
    da = torch.empty(B * T, 2 * C, device=a.device, dtype=da_dtype)
    dw = torch.empty(C, K, device=a.device, dtype=torch.float32)
    db = torch.empty(C, device=a.device, dtype=torch.float32)
    defer = side is not None
    L.call("cfm_glu_dwconv_bwd", L.ptr(dy), L.ptr(a), L.dt(a), L.ptr(w_dw), L.ptr(da), L.dt(da),
           None if defer else L.ptr(dw), None if defer else L.ptr(db), B, T, C, K, L.ptr(ws), L.stream())
    return _dwconv_wgrad(ws, B, T, C, K, da, dw, db, side)


def bn_silu_glu_dwconv_bwd(dz, y, gamma, beta, mean, invstd, training, a, w_dw, B, T, C, K, ws, da_dtype,
                           side=None, reduce_sums=None, world=1):
    """BatchNorm1d + SiLU backward folded into the GLU + depthwise-conv backward (cfm_glu_dwconv_bwd_bn): the
    BN parameter gradients come from cfm_bn_silu_bwd_sums, the BN input gradient is formed inside the depthwise
    kernel and never stored.  reduce_sums / world: SyncBatchNorm (as bn_silu_bwd_sync).
    Returns (da, dw_dw, db_dw, dgamma, dbeta)."""
    M = B * T
    dbg = torch.empty(2, C, device=y.device, dtype=torch.float32)     # [dbeta; dgamma] of this rank
    L.call("cfm_bn_silu_bwd_sums", L.ptr(dz), L.dt(dz), L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(mean),
           L.ptr(invstd), M, C, L.ptr(ws), L.ptr(dbg[0]), L.ptr(dbg[1]), L.stream())
    tot, rows = dbg, M
    if reduce_sums is not None and training:
        tot = dbg.clone()
        reduce_sums(tot)
        rows = int(world) * M
    da = torch.empty(M, 2 * C, device=a.device, dtype=da_dtype)
    dw = torch.empty(C, K, device=a.device, dtype=torch.float32)
    db = torch.empty(C, device=a.device, dtype=torch.float32)
    defer = side is not None
    L.call("cfm_glu_dwconv_bwd_bn", L.ptr(dz), L.dt(dz), L.ptr(y), L.ptr(gamma), L.ptr(beta), L.ptr(mean),
           L.ptr(invstd), L.ptr(tot[0]), L.ptr(tot[1]), 1.0 / rows, int(bool(training)), L.ptr(a), L.dt(a),
           L.ptr(w_dw), L.ptr(da), L.dt(da), None if defer else L.ptr(dw), None if defer else L.ptr(db), B, T, C, K,
           L.ptr(ws), L.stream())
    da, dw, db = _dwconv_wgrad(ws, B, T, C, K, da, dw, db, side)
    return da, dw, db, dbg[1], dbg[0]


def _dwconv_wgrad(ws, B, T, C, K, da, dw, db, side):
    defer = side is not None
    if defer:
        if getattr(side, "rgroup", None) is not None:
            np_ = L.load().cfm_convmod_nparts(B, T)
            dw, db = side.rgroup.add_dwconv(ws, np_, C, K, dw, db)
        else:
            side.run(lambda: L.call("cfm_glu_dwconv_bwd_wgrad", L.ptr(ws), B, T, C, K, L.ptr(dw), L.ptr(db),
                                    L.stream()), ws, dw, db)
    return da, dw, db


# ----------------------------------------------------------------------------- attention
def attn_fwd(qkv, lengths_i32, B, T, H, dk, pos=None, pos_u=None, pos_v=None, drop_p=0.0, seed=0):
    o = torch.empty(B * T, H * dk, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(B * H * T, device=qkv.device, dtype=torch.float32)
    L.call("cfm_attn_fwd", L.ptr(qkv), L.ptr(o), L.ptr(lse), L.ptr(lengths_i32), L.ptr(pos), L.ptr(pos_u),
           L.ptr(pos_v), B, T, H, dk, L.dt(qkv), float(drop_p), int(seed) & (2**64 - 1), L.stream())
    return o, lse


def attn_ws(B, T, H, dk, rel, device, dtype=torch.bfloat16):
    """A backward workspace (cfm_attn_bwd_ws_bytes) whose first B*H*T floats are the D slot: (ws, D view)."""
    ws = workspace(L.size_call("cfm_attn_bwd_ws_bytes", B, T, H, dk, int(rel), L.dt(torch.empty(0, dtype=dtype))),
                   device)
    return ws, ws[: B * H * T]


def attn_bwd(qkv, o, dout, lse, lengths_i32, B, T, H, dk, pos=None, pos_u=None, pos_v=None, drop_p=0.0, seed=0,
             D=None, ws=None, dpos_dtype=torch.float32):
    """D: optional (B*H*T,) fp32 rowsum(dO * O) per head, precomputed by the GEMM that produced dout
    (linear_dgrad(rowdot=...)); bf16 MFMA path only.  Rel-pos: D must be the head of ws (attn_ws).
    dpos_dtype: torch.bfloat16 returns dpos already in the compute dtype (rel-pos MFMA path, cfm_attn_bwd_ex)."""
    rel = pos is not None
    full = True     # ws is the whole cfm_attn_bwd_ws_bytes workspace (the non-rel whole-head path keeps dS^T there)
    if D is not None and ws is not None:
        if D.data_ptr() != ws.data_ptr():
            raise L.CfmError("attn_bwd: D must be the first B*H*T floats of ws")
    elif D is not None:
        if rel:
            raise L.CfmError("attn_bwd: rel-pos with a precomputed D needs its workspace (attn_ws)")
        ws = D
        full = False
    else:
        ws = workspace(L.size_call("cfm_attn_bwd_ws_bytes", B, T, H, dk, int(rel), L.dt(qkv)), qkv.device)
    dqkv = torch.empty_like(qkv)
    dpos = torch.empty(pos.shape, device=qkv.device, dtype=dpos_dtype) if rel else None
    dpu = torch.empty(H * dk, device=qkv.device, dtype=torch.float32) if rel else None
    dpv = torch.empty(H * dk, device=qkv.device, dtype=torch.float32) if rel else None
    d_ready = (1 if D is not None else 0) | (2 if full else 0)
    L.call("cfm_attn_bwd_ex", L.ptr(qkv), L.ptr(o), L.ptr(dout), L.ptr(lse), L.ptr(lengths_i32), L.ptr(pos),
           L.ptr(pos_u), L.ptr(pos_v), L.ptr(dqkv), L.ptr(dpos), L.dt(dpos), L.ptr(dpu), L.ptr(dpv), B, T, H, dk,
           L.dt(qkv), float(drop_p), int(seed) & (2**64 - 1), d_ready, L.ptr(ws), L.stream())
    return dqkv, dpos, dpu, dpv


# ----------------------------------------------------------------------------- conv subsampling
def conv1_fwd(x, w1, b1, out_dtype):
    B, F, T = x.shape
    C1 = w1.shape[0]
    F1, T1 = (F - 7) // 2 + 1, (T - 7) // 2 + 1
    h1 = torch.empty(B, F1, T1, C1, device=x.device, dtype=out_dtype)
    L.call("cfm_conv1_fwd", L.ptr(x), L.ptr(w1), L.ptr(b1), L.ptr(h1), L.dt(h1), B, F, T, C1, L.stream())
    return h1


def conv1_bwd_weight(dh1, x, C1):
    B, F, T = x.shape
    dw1 = torch.empty(C1, 49, device=x.device, dtype=torch.float32)
    db1 = torch.empty(C1, device=x.device, dtype=torch.float32)
    ws = workspace(L.size_call("cfm_conv1_bwd_ws_bytes", B, F, T, C1), x.device)
    L.call("cfm_conv1_bwd_weight", L.ptr(dh1), L.dt(dh1), L.ptr(x), L.ptr(dw1), L.ptr(db1), B, F, T, C1, L.ptr(ws),
           L.stream())
    return dw1, db1


def conv2_fwd(h1, w2r, b2, out_dtype):
    B, F1, T1, C1 = h1.shape
    C2 = w2r.shape[0]
    F2, T2 = (F1 - 3) // 2 + 1, (T1 - 3) // 2 + 1
    h2 = torch.empty(B, T2, F2, C2, device=h1.device, dtype=out_dtype)
    L.call("cfm_conv2_fwd", L.ptr(h1), L.ptr(w2r), L.ptr(b2), L.ptr(h2), L.dt(h2), L.dt(h1), B, F1, T1, C1, C2,
           L.stream())
    return h2


def conv2_bwd_data(dh2, w2r, F1, T1):
    B, T2, F2, C2 = dh2.shape
    C1 = w2r.shape[1] // 9
    dh1 = torch.empty(B, F1, T1, C1, device=dh2.device, dtype=dh2.dtype)
    if dh2.dtype == torch.bfloat16:     # LDS-DMA pipeline: gathered dh2 rows, packed K-major weights in ws
        ws = workspace(L.size_call("cfm_conv2_bwd_data_ws_bytes", C1, C2), dh2.device)
        L.call("cfm_conv2_bwd_data_ws", L.ptr(dh2), L.ptr(w2r), L.ptr(dh1), L.dt(dh2), B, F1, T1, C1, C2, L.ptr(ws),
               L.stream())
        return dh1
    L.call("cfm_conv2_bwd_data", L.ptr(dh2), L.ptr(w2r), L.ptr(dh1), L.dt(dh2), B, F1, T1, C1, C2, L.stream())
    return dh1


def conv2_bwd_weight(dh2, h1):
    B, F1, T1, C1 = h1.shape
    C2 = dh2.shape[-1]
    dw2r = torch.empty(C2, 9 * C1, device=h1.device, dtype=torch.float32)
    nb = L.size_call("cfm_conv2_bwd_weight_ws_bytes", B, F1, T1, C1, C2)
    ws = workspace(nb, h1.device) if nb else None     # deterministic split-K slabs (no atomics / memset)
    L.call("cfm_conv2_bwd_weight_ws", L.ptr(dh2), L.ptr(h1), L.ptr(dw2r), L.dt(h1), B, F1, T1, C1, C2, L.ptr(ws),
           L.stream())
    return dw2r


# ----------------------------------------------------------------------------- folded front-end
def ffold_geometry(B, F, T, C1, C2, D, k1, s1, k2, s2, dtype, hilo=True):
    """cfm_ffold_geometry (host only): the folded 'frame'-mode front-end's packed-input / GEMM geometry."""
    g = L.FfoldGeo(B=B, F=F, T=T, C1=C1, C2=C2, D=D, k1=k1, s1=s1, k2=k2, s2=s2,
                   dtype=BF16 if dtype == torch.bfloat16 else F32, hilo=int(bool(hilo)))
    L.call("cfm_ffold_geometry", L.ctypes.byref(g))
    return g


def ffold_pack(x, g, dtype):
    xt = torch.empty(g.xt_elems, device=x.device, dtype=dtype)
    L.call("cfm_ffold_pack", L.ptr(x), L.ptr(xt), L.ctypes.byref(g), L.stream())
    return xt


def ffold_compose(w1, b1, w2, b2, wp, bp, g, dtype):
    """-> (wfull (D, Kp) dtype, bfull (D) fp32, ws) -- ws keeps W_eff / b_eff for ffold_bwd_weights."""
    dev = w1.device
    wfull = torch.empty(g.D, g.Kp, device=dev, dtype=dtype)
    bfull = torch.empty(g.D, device=dev, dtype=torch.float32)
    ws = torch.empty(g.ws_floats, device=dev, dtype=torch.float32)
    L.call("cfm_ffold_compose", L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(wp), L.ptr(bp), L.ptr(wfull),
           L.ptr(bfull), L.ptr(ws), L.ctypes.byref(g), L.stream())
    return wfull, bfull, ws


def ffold_bwd_weights(H, S, w1, b1, w2, wp, ws, g):
    dw1, db1, dw2, db2, dwp = (torch.empty_like(t) for t in (w1, b1, w2, torch.empty(g.C2, device=w1.device), wp))
    L.call("cfm_ffold_bwd_weights", L.ptr(H), L.ptr(S), L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(wp), L.ptr(ws),
           L.ptr(dw1), L.ptr(db1), L.ptr(dw2), L.ptr(db2), L.ptr(dwp), L.ctypes.byref(g), L.stream())
    return dw1, db1, dw2, db2, dwp


# ----------------------------------------------------------------------------- CTC head
def _rows(x, batch_first):
    """(B, T, sb, st) of a (B, T, V) / (T, B, V) tensor with contiguous classes."""
    if x.stride(-1) != 1:
        raise L.CfmError("CTC: the class dimension must be contiguous")
    if batch_first:
        return x.shape[0], x.shape[1], x.stride(0), x.stride(1)
    return x.shape[1], x.shape[0], x.stride(1), x.stride(0)


def ctc_loss_fwd(x, targets_i32, ldt, tgt_off, in_len_i32, tgt_len_i32, smax, blank, zero_infinity, batch_first):
    """nll (B,) fp32 (0 where infinite and zero_infinity) + the workspace the backward needs."""
    B, T, sb, st = _rows(x, batch_first)
    V = x.shape[-1]
    ws = workspace(L.size_call("cfm_ctc_ws_bytes", B, T, smax), x.device)
    nll = torch.empty(B, device=x.device, dtype=torch.float32)
    L.call("cfm_ctc_loss_fwd", L.ptr(x), sb, st, L.ptr(targets_i32), ldt, L.ptr(tgt_off), L.ptr(in_len_i32),
           L.ptr(tgt_len_i32), B, T, V, smax, blank, int(bool(zero_infinity)), L.ptr(nll), L.ptr(ws), L.stream())
    return nll, ws


def ctc_mean(nll, tgt_len_i32, nonfinite=None):
    """torch.nn.CTCLoss reduction='mean' of nll (B,) as one launch -> 0-d fp32; nonfinite: optional (1,) int32
    device counter incremented when the result is not finite."""
    out = torch.empty((), device=nll.device, dtype=torch.float32)
    L.call("cfm_ctc_mean", L.ptr(nll), L.ptr(tgt_len_i32), nll.numel(), L.ptr(out), L.ptr(nonfinite), L.stream())
    return out


def ctc_loss_bwd(x, targets_i32, ldt, tgt_off, in_len_i32, tgt_len_i32, smax, blank, zero_infinity, batch_first, ws,
                 grad_out, reduction, grad_dtype=torch.float32):
    """d loss / d logits (softmax - posterior, scaled) in x's layout, dtype grad_dtype."""
    B, T, sb, st = _rows(x, batch_first)
    V = x.shape[-1]
    g = torch.empty(x.shape, device=x.device, dtype=grad_dtype)
    _, _, gsb, gst = _rows(g, batch_first)
    go = grad_out.float().contiguous()
    L.call("cfm_ctc_loss_bwd", L.ptr(x), sb, st, L.ptr(targets_i32), ldt, L.ptr(tgt_off), L.ptr(in_len_i32),
           L.ptr(tgt_len_i32), B, T, V, smax, blank, int(bool(zero_infinity)), L.ptr(ws), L.ptr(go),
           1 if go.numel() > 1 else 0, {"none": 0, "mean": 1, "sum": 2}[reduction], L.ptr(g), L.dt(g), gsb, gst,
           L.stream())
    return g


def ctc_greedy_decode(x, lengths_i32=None, blank=0, pad=-1, collapse=False, batch_first=True, compact=True):
    """argmax ids (B, T) int64 (torch.argmax semantics) and, if compact, the per-utterance id lists
    with `blank` / `pad` removed (and repeats collapsed if asked): (B, T) int32 padded with -1 + lengths."""
    B, T, sb, st = _rows(x, batch_first)
    ids = torch.empty(B, T, device=x.device, dtype=torch.int64)
    out = torch.empty(B, T, device=x.device, dtype=torch.int32) if compact else None
    out_len = torch.empty(B, device=x.device, dtype=torch.int32) if compact else None
    L.call("cfm_ctc_greedy_decode", L.ptr(x), sb, st, L.ptr(lengths_i32), B, T, x.shape[-1], int(blank), int(pad),
           int(bool(collapse)), L.ptr(ids), L.ptr(out), L.ptr(out_len), L.stream())
    return ids, out, out_len
