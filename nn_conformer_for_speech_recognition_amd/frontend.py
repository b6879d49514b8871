"""Encoder front-end and projection block on libcfm (autograd nodes over the C ABI).

  conv_subsample   lib/convsubsampling.py:16-45 — Conv2d(1->C1, 7x7, s2) -> Conv2d(C1->C2, 3x3, s2),
                   no activation/padding.  conv1 is a direct HBM-bound kernel writing NHWC; conv2 is
                   an implicit GEMM on MFMA that writes (B, T2, F2, C2) "frame-major" rows.
  linear           torch.nn.Linear (+ fused SiLU / dropout epilogue) — standard_linear (asrnn.py:208),
                   the per-frame projection, projection_fc.
  frame_frontend   'frame' projection mode: conv_subsample + the per-frame Linear folded into ONE GEMM over a
                   strided view of the packed mels (the three maps are linear with nothing between them).
  projection_block asrnn.py:73-89 — Linear -> SiLU -> BatchNorm1d (train: batch statistics).
"""
from __future__ import annotations

import os

import torch

from . import ops
from ._lib import ACT_NONE, ACT_SILU


def _cd(t, cd):
    return t if t.dtype == cd else ops.cast(t, cd)


class _ConvSubFn(torch.autograd.Function):
    """x (B, F, T) fp32 -> h2 (B, T2, F2, C2) in the compute dtype.  No input gradient (mels are data)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, cd):
        C1, C2 = w1.shape[0], w2.shape[0]
        h1 = ops.conv1_fwd(x, w1.reshape(C1, 49), b1, cd)
        w2r = _cd(w2.permute(0, 2, 3, 1).reshape(C2, 9 * C1).contiguous(), cd)   # [c2][kh][kw][c1]
        h2 = ops.conv2_fwd(h1, w2r, b2, cd)
        ctx.save_for_backward(x, h1, w2r)
        ctx.shapes = (C1, C2)
        return h2

    @staticmethod
    def backward(ctx, dh2):
        x, h1, w2r = ctx.saved_tensors
        C1, C2 = ctx.shapes
        dh2 = dh2.contiguous()
        if dh2.dtype != h1.dtype:
            dh2 = ops.cast(dh2, h1.dtype)
        B, F1, T1, _ = h1.shape
        dw2r = ops.conv2_bwd_weight(dh2, h1)
        db2 = ops.colsum(dh2.view(-1, C2))
        dh1 = ops.conv2_bwd_data(dh2, w2r, F1, T1)
        dw1, db1 = ops.conv1_bwd_weight(dh1, x, C1)
        dw2 = dw2r.view(C2, 3, 3, C1).permute(0, 3, 1, 2).contiguous()
        return None, dw1.view(C1, 1, 7, 7), db1, dw2, db2, None


def conv_subsample(x, w1, b1, w2, b2, cd):
    return _ConvSubFn.apply(x, w1, b1, w2, b2, cd)


class _FrameFoldFn(torch.autograd.Function):
    """x (B, F, T) fp32 -> drop(Linear(flatten_frames(ConvSubSampling(x)))) (B*T2, D) fp32 as ONE GEMM over
    a strided view of the packed mels (frontfold.hip; the fold of convsubsampling.py:41-43 + asrnn.py:208).
    No input gradient (mels are data)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, wp, bp, cd, s1, s2, drop_p, seed, hilo):
        B, F, T = x.shape
        D = wp.shape[0]
        g = ops.ffold_geometry(B, F, T, w1.shape[0], w2.shape[0], D, w1.shape[-1], s1, w2.shape[-1], s2, cd, hilo)
        if wp.shape[1] != g.F2 * g.C2:
            raise ValueError(f"projection expects {wp.shape[1]} features, the front-end gives {g.F2 * g.C2}")
        xt = ops.ffold_pack(x, g, cd)
        wfull, bfull, ws = ops.ffold_compose(w1, b1, w2, b2, wp, bp, g, cd)
        h = torch.empty(B * g.T2, D, device=x.device, dtype=torch.float32)
        ops.gemm(xt, wfull, h, g.T2, D, g.Kp, lda=g.lda, stride_a=g.Tslot * g.Cx, batch=B, stride_c=g.T2 * D,
                 bias=bfull, drop_p=drop_p, seed=seed, allow_overlap=True)
        ctx.save_for_backward(xt, ws, w1, b1, w2, wp)
        ctx.g = g
        ctx.cfg = (cd, drop_p, seed)
        return h

    @staticmethod
    def backward(ctx, dh):
        xt, ws, w1, b1, w2, wp = ctx.saved_tensors
        g = ctx.g
        cd, drop_p, seed = ctx.cfg
        B, T2, T2p, D = g.B, g.T2, g.T2p, g.D
        dh = dh.contiguous()
        gr = ops.scale_dropout(dh, 1.0, drop_p, seed, 0, out_dtype=cd) if drop_p > 0 else _cd(dh, cd)
        # the gradient in the view's slot layout: T2 rows per utterance, the padding rows past T2 zero (a fresh
        # buffer per backward: no state shared between models, streams or shapes)
        gpad = torch.empty(B, T2p, D, device=dh.device, dtype=cd)
        gpad[:, T2:].zero_()
        gpad[:, :T2].copy_(gr.view(B, T2, D))
        K = B * T2p
        H = torch.empty(D, g.Kp, device=dh.device, dtype=torch.float32)
        split = max(2, min(16, K // 512))      # >= 2: the slab path (deterministic) also yields S = colsum(G)
        if cd == torch.bfloat16:
            S = torch.empty(D, device=dh.device, dtype=torch.float32)
            wsk = ops.workspace(4 * (split * D * g.Kp + split * D), dh.device)
            ops.gemm(gpad.view(K, D), xt, H, D, g.Kp, K, a_kmajor=False, lda=D, b_kmajor=False, ldb=g.lda,
                     split_k=split, workspace=wsk, a_colsum=S, allow_overlap=True)
        else:
            wsk = ops.workspace(4 * split * D * g.Kp, dh.device)
            ops.gemm(gpad.view(K, D), xt, H, D, g.Kp, K, a_kmajor=False, lda=D, b_kmajor=False, ldb=g.lda,
                     split_k=split, workspace=wsk, allow_overlap=True)
            S = ops.colsum(gpad.view(K, D))
        dw1, db1, dw2, db2, dwp = ops.ffold_bwd_weights(H, S, w1, b1, w2, wp, ws, g)
        return None, dw1, db1, dw2, db2, dwp, S, None, None, None, None, None, None


def frame_frontend(convsub, proj, x, cd, drop_p=0.0, seed=0, hilo=True):
    """The 'frame'-mode encoder input: dropout(proj(ConvSubSampling(x) per frame)) -> (B*T2, D) fp32.
    convsub: lib.convsubsampling.ConvSubSampling; proj: the nn.Linear(F2*C2, D) (features (f2, c2)).
    x (B, 1, F, T) or (B, F, T) mels.  Folded into one GEMM (frontfold.hip) unless CFM_FFOLD=0 (the unfolded
    conv1 -> conv2 -> Linear kernels, for A/B)."""
    if x.dim() == 4:
        x = x.reshape(x.shape[0], x.shape[2], x.shape[3])
    x = x.float().contiguous()
    c1, c2 = convsub.conv_sub_1, convsub.conv_sub_2
    if os.environ.get("CFM_FFOLD", "1") == "0":
        h2 = convsub.forward_frames(x, cd)
        B, T2 = h2.shape[0], h2.shape[1]
        return linear(h2.reshape(B * T2, -1), proj.weight, proj.bias, cd=cd, drop_p=drop_p, seed=seed)
    convsub._check()
    return _FrameFoldFn.apply(x, c1.weight, c1.bias, c2.weight, c2.bias, proj.weight, proj.bias, cd,
                              int(c1.stride[0]), int(c2.stride[0]), float(drop_p), int(seed), bool(hilo))


class _LinearFn(torch.autograd.Function):
    """y = drop(act(x·Wᵀ + b)) with x (M, K) in the compute dtype, W fp32 master; y in out_dtype."""

    @staticmethod
    def forward(ctx, x, w, b, cd, act, drop_p, seed, out_dtype):
        xc = _cd(x, cd)
        wc = _cd(w, cd)
        pre = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=cd) if act == ACT_SILU else None
        y = ops.linear(xc, wc, b, out_dtype=out_dtype, act=act, pre=pre, drop_p=drop_p, seed=seed)
        ctx.save_for_backward(xc, wc, pre)
        ctx.cfg = (cd, act, drop_p, seed, x.dtype, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc, pre = ctx.saved_tensors
        cd, act, drop_p, seed, xdt, has_b = ctx.cfg
        dy = dy.contiguous()
        if act == ACT_SILU or drop_p > 0:
            g = ops.scale_dropout(dy, 1.0, drop_p, seed, 0, out_dtype=cd)
            if act == ACT_SILU:
                g = ops.silu_bwd(g, pre, out_dtype=cd)
        else:
            g = dy if dy.dtype == cd else ops.cast(dy, cd)
        dw = ops.linear_wgrad(g, xc)
        db = ops.colsum(g) if has_b else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = ops.linear_dgrad(g, wc, out_dtype=xdt)
        return dx, dw, db, None, None, None, None, None


def linear(x, w, b=None, cd=torch.bfloat16, act=ACT_NONE, drop_p=0.0, seed=0, out_dtype=torch.float32):
    return _LinearFn.apply(x, w, b, cd, act, float(drop_p), int(seed), out_dtype)


class _BatchNormFn(torch.autograd.Function):
    """BatchNorm1d over rows of (M, C) fp32 (asrnn.py:88 projection_batch_norm)."""

    @staticmethod
    def forward(ctx, y, gamma, beta, rm, rv, momentum, eps, training):
        z, mean, invstd = ops.bn_fwd(y, gamma, beta, rm, rv, momentum, eps, training, act=0)
        ctx.save_for_backward(y, gamma, beta, mean, invstd)
        ctx.training = training
        return z

    @staticmethod
    def backward(ctx, dz):
        y, gamma, beta, mean, invstd = ctx.saved_tensors
        dy, dg, db = ops.bn_bwd(dz.contiguous(), y, gamma, beta, mean, invstd, ctx.training, act=0)
        return dy, dg, db, None, None, None, None, None


def batch_norm(y, bn, training):
    if training and bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
    mom = bn.momentum if bn.momentum is not None else 0.1
    return _BatchNormFn.apply(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, mom, bn.eps, training)


def projection_block(x, fc, bn, training, cd):
    """asrnn.py:73-89: Linear -> SiLU -> BatchNorm1d on (M, d)."""
    s = linear(x, fc.weight, fc.bias, cd=cd, act=ACT_SILU, out_dtype=torch.float32)
    return batch_norm(s, bn, training)
