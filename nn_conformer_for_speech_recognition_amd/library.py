"""torch.library registration of the libcfm hot ops: ``torch.ops.cfm.*``.

Each op is a PyTorch custom operator over the C ABI (include/cfm.h) with
  * a CUDA(HIP) kernel only -- CPU tensors raise (no fallback), like every other libcfm entry point;
  * a fake (meta) kernel, so FakeTensor / AOTAutograd / torch.compile can trace it;
  * an autograd formula whose backward is itself a cfm op (traceable end to end).

Ops (SURVEY.md §3.3 block; the reference reaches them through torchaudio.models.Conformer at
/root/reference/lib/standard/asrnn.py:29,214 and torch.nn.functional.ctc_loss at runner.py:143):
  cfm::gemm                       C = A·Bᵀ in either operand layout (no autograd)
  cfm::linear / linear_bwd        y = out_scale * dropout(x·wᵀ + b) + residual
  cfm::linear_silu / _bwd         y = dropout(silu(x·wᵀ + b)), pre-activation returned for the backward
  cfm::layer_norm / _bwd          (y, mean, rstd) over the last dim
  cfm::attention / _bwd           key-padding-masked multi-head attention core on packed [q|k|v] rows
  cfm::attention_rel / _bwd       the same with Transformer-XL relative positions (projected table pos, biases u / v:
                                  transformers modeling_wav2vec2_conformer.py:528-565, the rel-pos MFMA kernels)
  cfm::conv_glu_dwconv_bn_silu / _bwd   GLU -> depthwise Conv1d -> BatchNorm1d -> SiLU of the ConvModule
  cfm::ctc_loss / _bwd            per-utterance CTC negative log-likelihood (log-probs, batch-first)

`layer_forward` composes them into one torchaudio ConformerLayer; Conformer.forward takes that route
while torch.compile traces it (conformer.py), so the encoder compiles with fullgraph=True.  The eager /
HIP-graph training path keeps the fused single-node layer (grouped weight gradients, side streams).
Dropout masks are counter-based (seed + element index, cfm_common.h); bind a device step counter with
cfm_rng_bind (as bench.py does for graph replay) for fresh masks per compiled step.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor

from . import ops
from . import _lib as L

_EPS = 1e-5


# ----------------------------------------------------------------------------- GEMM
@torch.library.custom_op("cfm::gemm", mutates_args=(), device_types="cuda")
def gemm(a: Tensor, b: Tensor, a_kmajor: bool, b_kmajor: bool, out_dtype: torch.dtype) -> Tensor:
    """C (M, N) = A·Bᵀ; A is (M, K) if a_kmajor else (K, M); B is (N, K) if b_kmajor else (K, N)."""
    M, K = a.shape if a_kmajor else (a.shape[1], a.shape[0])
    N = b.shape[0] if b_kmajor else b.shape[1]
    c = torch.empty(M, N, device=a.device, dtype=out_dtype)
    return ops.gemm(a.contiguous(), b.contiguous(), c, M, N, K, a_kmajor=a_kmajor, b_kmajor=b_kmajor)


@gemm.register_fake
def _(a, b, a_kmajor, b_kmajor, out_dtype):
    M = a.shape[0] if a_kmajor else a.shape[1]
    N = b.shape[0] if b_kmajor else b.shape[1]
    return a.new_empty(M, N, dtype=out_dtype)


# ----------------------------------------------------------------------------- linear (+ epilogues)
# The weight may be the fp32 master: it is cast to x's (compute) dtype inside the op, so its gradient stays
# an fp32 GEMM output (a .to(bf16) in front of the op would round dW through bf16 on the way back).
def _wc(w, x):
    w = w.contiguous()
    return w if w.dtype == x.dtype else ops.cast(w, x.dtype)


@torch.library.custom_op("cfm::linear", mutates_args=(), device_types="cuda")
def linear(x: Tensor, w: Tensor, bias: Optional[Tensor], residual: Optional[Tensor], drop_p: float, seed: int,
           out_scale: float, out_dtype: torch.dtype) -> Tensor:
    return ops.linear(x.contiguous(), _wc(w, x), bias, out_dtype=out_dtype, drop_p=drop_p, seed=seed,
                      out_scale=out_scale, residual=residual.contiguous() if residual is not None else None)


@linear.register_fake
def _(x, w, bias, residual, drop_p, seed, out_scale, out_dtype):
    return x.new_empty(x.shape[0], w.shape[0], dtype=out_dtype)


@torch.library.custom_op("cfm::linear_bwd", mutates_args=(), device_types="cuda")
def linear_bwd(gy: Tensor, x: Tensor, w: Tensor, drop_p: float, seed: int, out_scale: float
               ) -> tuple[Tensor, Tensor, Tensor]:
    """(dx, dw fp32, db fp32) of cfm::linear: the dropout mask is regenerated from (seed, element index)."""
    g = ops.scale_dropout(gy.contiguous(), out_scale, drop_p, seed, 0, out_dtype=x.dtype)
    dx = ops.linear_dgrad(g, _wc(w, x))
    db = torch.empty(w.shape[0], device=x.device, dtype=torch.float32)
    dw = ops.linear_wgrad(g, x.contiguous(), bias_out=db)
    return dx, dw, db


@linear_bwd.register_fake
def _(gy, x, w, drop_p, seed, out_scale):
    return (x.new_empty(x.shape), w.new_empty(w.shape, dtype=torch.float32),
            w.new_empty(w.shape[0], dtype=torch.float32))


def _linear_setup(ctx, inputs, output):
    x, w, bias, residual, drop_p, seed, out_scale, _ = inputs
    ctx.save_for_backward(x, w)
    ctx.cfg = (drop_p, seed, out_scale, bias is not None, residual is not None)


def _linear_backward(ctx, gy):
    x, w = ctx.saved_tensors
    drop_p, seed, out_scale, has_b, has_r = ctx.cfg
    dx, dw, db = torch.ops.cfm.linear_bwd(gy, x, w, drop_p, seed, out_scale)
    return dx, dw.to(w.dtype), db if has_b else None, gy if has_r else None, None, None, None, None


linear.register_autograd(_linear_backward, setup_context=_linear_setup)


@torch.library.custom_op("cfm::linear_silu", mutates_args=(), device_types="cuda")
def linear_silu(x: Tensor, w: Tensor, bias: Optional[Tensor], drop_p: float, seed: int) -> tuple[Tensor, Tensor]:
    """(y, pre): y = dropout(silu(pre)), pre = x·wᵀ + b, both in x's dtype (one GEMM, fused epilogue)."""
    x, w = x.contiguous(), _wc(w, x)
    pre = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=x.dtype)
    y = ops.linear(x, w, bias, act=L.ACT_SILU, pre=pre, drop_p=drop_p, seed=seed)
    return y, pre


@linear_silu.register_fake
def _(x, w, bias, drop_p, seed):
    return x.new_empty(x.shape[0], w.shape[0]), x.new_empty(x.shape[0], w.shape[0])


@torch.library.custom_op("cfm::linear_silu_bwd", mutates_args=(), device_types="cuda")
def linear_silu_bwd(gy: Tensor, x: Tensor, w: Tensor, pre: Tensor, drop_p: float, seed: int
                    ) -> tuple[Tensor, Tensor, Tensor]:
    g = ops.scale_dropout(gy.contiguous(), 1.0, drop_p, seed, 0, out_dtype=x.dtype)
    gp = ops.silu_bwd(g, pre)
    dx = ops.linear_dgrad(gp, _wc(w, x))
    db = torch.empty(w.shape[0], device=x.device, dtype=torch.float32)
    dw = ops.linear_wgrad(gp, x.contiguous(), bias_out=db)
    return dx, dw, db


@linear_silu_bwd.register_fake
def _(gy, x, w, pre, drop_p, seed):
    return (x.new_empty(x.shape), w.new_empty(w.shape, dtype=torch.float32),
            w.new_empty(w.shape[0], dtype=torch.float32))


def _linear_silu_setup(ctx, inputs, output):
    x, w, bias, drop_p, seed = inputs
    ctx.save_for_backward(x, w, output[1])
    ctx.cfg = (drop_p, seed, bias is not None)


def _linear_silu_backward(ctx, gy, _gpre):
    x, w, pre = ctx.saved_tensors
    drop_p, seed, has_b = ctx.cfg
    dx, dw, db = torch.ops.cfm.linear_silu_bwd(gy, x, w, pre, drop_p, seed)
    return dx, dw.to(w.dtype), db if has_b else None, None, None


linear_silu.register_autograd(_linear_silu_backward, setup_context=_linear_silu_setup)


# ----------------------------------------------------------------------------- LayerNorm
@torch.library.custom_op("cfm::layer_norm", mutates_args=(), device_types="cuda")
def layer_norm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float, out_dtype: torch.dtype
               ) -> tuple[Tensor, Tensor, Tensor]:
    """(y (M, D) out_dtype, mean (M,), rstd (M,)) of x (M, D)."""
    return ops.layernorm_fwd(x.contiguous(), gamma, beta, eps, out_dtype=out_dtype)


@layer_norm.register_fake
def _(x, gamma, beta, eps, out_dtype):
    M = x.shape[0]
    return x.new_empty(x.shape, dtype=out_dtype), x.new_empty(M, dtype=torch.float32), \
        x.new_empty(M, dtype=torch.float32)


@torch.library.custom_op("cfm::layer_norm_bwd", mutates_args=(), device_types="cuda")
def layer_norm_bwd(dy: Tensor, x: Tensor, gamma: Tensor, mean: Tensor, rstd: Tensor
                   ) -> tuple[Tensor, Tensor, Tensor]:
    dx, dg, db = ops.layernorm_bwd(dy.contiguous(), x.contiguous(), gamma, mean, rstd, dx_dtype=x.dtype)
    return dx, dg.clone(), db.clone()       # (dgamma, dbeta are rows of one buffer: outputs must not alias)


@layer_norm_bwd.register_fake
def _(dy, x, gamma, mean, rstd):
    D = x.shape[1]
    return x.new_empty(x.shape), x.new_empty(D, dtype=torch.float32), x.new_empty(D, dtype=torch.float32)


def _ln_setup(ctx, inputs, output):
    x, gamma, _, _, _ = inputs
    ctx.save_for_backward(x, gamma, output[1], output[2])


def _ln_backward(ctx, gy, _gm, _gr):
    x, gamma, mean, rstd = ctx.saved_tensors
    dx, dg, db = torch.ops.cfm.layer_norm_bwd(gy, x, gamma, mean, rstd)
    return dx, dg.to(gamma.dtype), db.to(gamma.dtype), None, None


layer_norm.register_autograd(_ln_backward, setup_context=_ln_setup)


# ----------------------------------------------------------------------------- attention
@torch.library.custom_op("cfm::attention", mutates_args=(), device_types="cuda")
def attention(qkv: Tensor, lengths: Tensor, B: int, T: int, H: int, drop_p: float, seed: int
              ) -> tuple[Tensor, Tensor]:
    """(o (B*T, H*dk), lse (B*H*T,) fp32) from qkv (B*T, 3*H*dk) rows [q | k | v]; lengths (B,) int32."""
    dk = qkv.shape[1] // (3 * H)
    return ops.attn_fwd(qkv.contiguous(), lengths.to(torch.int32).contiguous(), B, T, H, dk, drop_p=drop_p,
                        seed=seed)


@attention.register_fake
def _(qkv, lengths, B, T, H, drop_p, seed):
    return qkv.new_empty(qkv.shape[0], qkv.shape[1] // 3), qkv.new_empty(B * H * T, dtype=torch.float32)


@torch.library.custom_op("cfm::attention_bwd", mutates_args=(), device_types="cuda")
def attention_bwd(qkv: Tensor, o: Tensor, do: Tensor, lse: Tensor, lengths: Tensor, B: int, T: int, H: int,
                  drop_p: float, seed: int) -> Tensor:
    dk = qkv.shape[1] // (3 * H)
    dqkv, _, _, _ = ops.attn_bwd(qkv.contiguous(), o.contiguous(), do.contiguous(), lse,
                                 lengths.to(torch.int32).contiguous(), B, T, H, dk, drop_p=drop_p, seed=seed)
    return dqkv


@attention_bwd.register_fake
def _(qkv, o, do, lse, lengths, B, T, H, drop_p, seed):
    return qkv.new_empty(qkv.shape)


def _attn_setup(ctx, inputs, output):
    qkv, lengths, B, T, H, drop_p, seed = inputs
    ctx.save_for_backward(qkv, lengths, output[0], output[1])
    ctx.cfg = (B, T, H, drop_p, seed)


def _attn_backward(ctx, go, _glse):
    qkv, lengths, o, lse = ctx.saved_tensors
    B, T, H, drop_p, seed = ctx.cfg
    dqkv = torch.ops.cfm.attention_bwd(qkv, o, go.to(qkv.dtype), lse, lengths, B, T, H, drop_p, seed)
    return dqkv, None, None, None, None, None, None


attention.register_autograd(_attn_backward, setup_context=_attn_setup)


# ----------------------------------------------------------------------------- relative-position attention
@torch.library.custom_op("cfm::attention_rel", mutates_args=(), device_types="cuda")
def attention_rel(qkv: Tensor, pos: Tensor, pos_u: Tensor, pos_v: Tensor, lengths: Tensor, B: int, T: int, H: int,
                  drop_p: float, seed: int) -> tuple[Tensor, Tensor]:
    """(o, lse) of relative-position attention: scores scale * ((q+u)·k_j + (q+v)·pos[T-1-i+j]); pos (2T-1, H*dk)
    in qkv's dtype (the projected table linear_pos(pe)), pos_u / pos_v (H*dk,) fp32."""
    dk = qkv.shape[1] // (3 * H)
    return ops.attn_fwd(qkv.contiguous(), lengths.to(torch.int32).contiguous(), B, T, H, dk, pos.contiguous(),
                        pos_u.float().contiguous(), pos_v.float().contiguous(), drop_p=drop_p, seed=seed)


@attention_rel.register_fake
def _(qkv, pos, pos_u, pos_v, lengths, B, T, H, drop_p, seed):
    return qkv.new_empty(qkv.shape[0], qkv.shape[1] // 3), qkv.new_empty(B * H * T, dtype=torch.float32)


@torch.library.custom_op("cfm::attention_rel_bwd", mutates_args=(), device_types="cuda")
def attention_rel_bwd(qkv: Tensor, o: Tensor, do: Tensor, lse: Tensor, pos: Tensor, pos_u: Tensor, pos_v: Tensor,
                      lengths: Tensor, B: int, T: int, H: int, drop_p: float, seed: int
                      ) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    """(dqkv, dpos in pos's dtype, dpos_u, dpos_v fp32)."""
    dk = qkv.shape[1] // (3 * H)
    dpos_dt = torch.bfloat16 if pos.dtype == torch.bfloat16 else torch.float32
    dqkv, dpos, dpu, dpv = ops.attn_bwd(qkv.contiguous(), o.contiguous(), do.contiguous(), lse,
                                        lengths.to(torch.int32).contiguous(), B, T, H, dk, pos.contiguous(),
                                        pos_u.float().contiguous(), pos_v.float().contiguous(), drop_p=drop_p,
                                        seed=seed, dpos_dtype=dpos_dt)
    return dqkv, dpos.to(pos.dtype), dpu, dpv


@attention_rel_bwd.register_fake
def _(qkv, o, do, lse, pos, pos_u, pos_v, lengths, B, T, H, drop_p, seed):
    return (qkv.new_empty(qkv.shape), pos.new_empty(pos.shape), pos_u.new_empty(pos_u.shape, dtype=torch.float32),
            pos_v.new_empty(pos_v.shape, dtype=torch.float32))


def _attn_rel_setup(ctx, inputs, output):
    qkv, pos, pos_u, pos_v, lengths, B, T, H, drop_p, seed = inputs
    ctx.save_for_backward(qkv, pos, pos_u, pos_v, lengths, output[0], output[1])
    ctx.cfg = (B, T, H, drop_p, seed)


def _attn_rel_backward(ctx, go, _glse):
    qkv, pos, pos_u, pos_v, lengths, o, lse = ctx.saved_tensors
    B, T, H, drop_p, seed = ctx.cfg
    dqkv, dpos, dpu, dpv = torch.ops.cfm.attention_rel_bwd(qkv, o, go.to(qkv.dtype), lse, pos, pos_u, pos_v, lengths,
                                                           B, T, H, drop_p, seed)
    return dqkv, dpos, dpu.to(pos_u.dtype), dpv.to(pos_v.dtype), None, None, None, None, None, None


attention_rel.register_autograd(_attn_rel_backward, setup_context=_attn_rel_setup)


def _rel_table(T, d, device, dtype):
    """The (2T-1, d) sinusoid of conformer.rel_pos_table (the same host ops, so the same values), as traceable
    torch ops, cast to the compute dtype."""
    import math
    pos = torch.arange(T - 1, -T, -1, dtype=torch.int64).float().unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.int64).float() * -(math.log(10000.0) / d))
    pe = torch.zeros(2 * T - 1, d)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.to(device=device, dtype=dtype)


# ----------------------------------------------------------------------------- ConvModule middle
@torch.library.custom_op("cfm::conv_glu_dwconv_bn_silu", mutates_args=(), device_types="cuda")
def conv_glu_dwconv_bn_silu(a: Tensor, w_dw: Tensor, b_dw: Tensor, gamma: Tensor, beta: Tensor,
                            running_mean: Optional[Tensor], running_var: Optional[Tensor], training: bool,
                            eps: float, B: int, out_dtype: torch.dtype) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    """ConvModule GLU -> depthwise Conv1d(K, 'same') -> BatchNorm1d -> SiLU on token-major a (B*T, 2C).
    Returns (z (B*T, C) out_dtype, y (B*T, C) fp32 BN input, mean (C,), invstd (C,)).  training: batch
    statistics (the running-stat update is the caller's: this op mutates nothing); else running_mean /
    running_var are read."""
    M, C2 = a.shape
    C, K = w_dw.shape
    T = M // B
    ws = ops.convmod_ws(B, T, C, K, a.device)
    y = ops.glu_dwconv_fwd(a.contiguous(), w_dw.contiguous(), b_dw, B, T, C, K, ws)
    if training:
        z, mean, invstd = ops.bn_silu_fwd(y, gamma, beta, None, None, 0.0, eps, True, B, T, C, ws, out_dtype)
    else:
        z, mean, invstd = ops.bn_silu_fwd(y, gamma, beta, running_mean, running_var, 0.0, eps, False, B, T, C, ws,
                                          out_dtype)
    return z, y, mean, invstd


@conv_glu_dwconv_bn_silu.register_fake
def _(a, w_dw, b_dw, gamma, beta, running_mean, running_var, training, eps, B, out_dtype):
    M = a.shape[0]
    C = w_dw.shape[0]
    f = torch.float32
    return a.new_empty(M, C, dtype=out_dtype), a.new_empty(M, C, dtype=f), a.new_empty(C, dtype=f), \
        a.new_empty(C, dtype=f)


@torch.library.custom_op("cfm::conv_glu_dwconv_bn_silu_bwd", mutates_args=(), device_types="cuda")
def conv_glu_dwconv_bn_silu_bwd(dz: Tensor, a: Tensor, y: Tensor, w_dw: Tensor, gamma: Tensor, beta: Tensor,
                                mean: Tensor, invstd: Tensor, training: bool, B: int
                                ) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(da, dw_dw (C, K), db_dw, dgamma, dbeta), the BN input gradient folded into the depthwise backward."""
    M = a.shape[0]
    C, K = w_dw.shape
    T = M // B
    a, dz, w_dw = a.contiguous(), dz.contiguous(), w_dw.contiguous()
    ws = ops.convmod_ws(B, T, C, K, a.device)
    if K in ops.BN_FOLD_K:
        da, dw, db, dg, dbt = ops.bn_silu_glu_dwconv_bwd(dz, y, gamma, beta, mean, invstd, training, a, w_dw, B, T,
                                                          C, K, ws, a.dtype)
    else:
        dy, dg, dbt = ops.bn_silu_bwd(dz, y, gamma, beta, mean, invstd, training, ws)
        da, dw, db = ops.glu_dwconv_bwd(dy, a, w_dw, B, T, C, K, ws, a.dtype)
    return da, dw, db, dg.clone(), dbt.clone()


@conv_glu_dwconv_bn_silu_bwd.register_fake
def _(dz, a, y, w_dw, gamma, beta, mean, invstd, training, B):
    C = w_dw.shape[0]
    f = torch.float32
    return a.new_empty(a.shape), w_dw.new_empty(w_dw.shape, dtype=f), a.new_empty(C, dtype=f), \
        a.new_empty(C, dtype=f), a.new_empty(C, dtype=f)


def _conv_setup(ctx, inputs, output):
    a, w_dw, _, gamma, beta, _, _, training, _, B, _ = inputs
    ctx.save_for_backward(a, w_dw, gamma, beta, output[1], output[2], output[3])
    ctx.cfg = (training, B)


def _conv_backward(ctx, gz, _gy, _gm, _gi):
    a, w_dw, gamma, beta, y, mean, invstd = ctx.saved_tensors
    training, B = ctx.cfg
    da, dw, db, dg, dbt = torch.ops.cfm.conv_glu_dwconv_bn_silu_bwd(gz, a, y, w_dw, gamma, beta, mean, invstd,
                                                                     training, B)
    return da, dw.to(w_dw.dtype), db, dg, dbt, None, None, None, None, None, None


conv_glu_dwconv_bn_silu.register_autograd(_conv_backward, setup_context=_conv_setup)


# ----------------------------------------------------------------------------- CTC
@torch.library.custom_op("cfm::ctc_loss", mutates_args=(), device_types="cuda")
def ctc_loss(log_probs: Tensor, targets: Tensor, input_lengths: Tensor, target_lengths: Tensor, blank: int,
             zero_infinity: bool) -> Tensor:
    """nll (B,) fp32 of log_probs (B, T, V) fp32 (batch-first, classes contiguous) against padded targets
    (B, S) -- torch.nn.functional.ctc_loss(reduction='none') semantics."""
    x = log_probs.contiguous()
    tg = targets.to(torch.int32).contiguous()
    il = input_lengths.to(torch.int32).contiguous()
    tl = target_lengths.to(torch.int32).contiguous()
    nll, _ = ops.ctc_loss_fwd(x, tg, tg.shape[1], None, il, tl, tg.shape[1], blank, zero_infinity, True)
    return nll


@ctc_loss.register_fake
def _(log_probs, targets, input_lengths, target_lengths, blank, zero_infinity):
    return log_probs.new_empty(log_probs.shape[0], dtype=torch.float32)


@torch.library.custom_op("cfm::ctc_loss_bwd", mutates_args=(), device_types="cuda")
def ctc_loss_bwd(gnll: Tensor, log_probs: Tensor, targets: Tensor, input_lengths: Tensor, target_lengths: Tensor,
                 blank: int, zero_infinity: bool) -> Tensor:
    """d Σ_b gnll[b]·nll[b] / d log_probs (the forward recursion is re-run for its workspace)."""
    x = log_probs.contiguous()
    tg = targets.to(torch.int32).contiguous()
    il = input_lengths.to(torch.int32).contiguous()
    tl = target_lengths.to(torch.int32).contiguous()
    S = tg.shape[1]
    _, ws = ops.ctc_loss_fwd(x, tg, S, None, il, tl, S, blank, zero_infinity, True)
    g = gnll.float().contiguous()
    if g.numel() == 1:
        g = g.expand(x.shape[0]).contiguous()
    return ops.ctc_loss_bwd(x, tg, S, None, il, tl, S, blank, zero_infinity, True, ws, g, "none")


@ctc_loss_bwd.register_fake
def _(gnll, log_probs, targets, input_lengths, target_lengths, blank, zero_infinity):
    return log_probs.new_empty(log_probs.shape)


def _ctc_setup(ctx, inputs, output):
    log_probs, targets, il, tl, blank, zi = inputs
    ctx.save_for_backward(log_probs, targets, il, tl)
    ctx.cfg = (blank, zi)


def _ctc_backward(ctx, g):
    log_probs, targets, il, tl = ctx.saved_tensors
    blank, zi = ctx.cfg
    return torch.ops.cfm.ctc_loss_bwd(g, log_probs, targets, il, tl, blank, zi), None, None, None, None, None


ctc_loss.register_autograd(_ctc_backward, setup_context=_ctc_setup)


# ----------------------------------------------------------------------------- one ConformerLayer from the ops
def layer_forward(layer, x, lens, B, T, cd, seed):
    """torchaudio ConformerLayer.forward on x (B*T, d) fp32 token-major, composed of
    torch.ops.cfm.* so FakeTensor / AOTAutograd / torch.compile(fullgraph=True) trace it.  Same kernels,
    seeds and dropout placement as the fused node in conformer.py; pos_enc='rel' projects the positional table per
    layer (cfm::linear, dW_pos through its backward) and runs cfm::attention_rel."""
    cfm = torch.ops.cfm
    P = layer.params()
    R = P[30:]            # rel-pos: linear_pos.weight, pos_bias_u, pos_bias_v (conformer._REL_PNAMES)
    p = float(layer.dropout) if layer.training else 0.0
    d, H, K = layer.d, layer.H, layer.K
    f32 = torch.float32

    def ffn(x, o, s):
        xn, _, _ = cfm.layer_norm(x, P[o], P[o + 1], _EPS, cd)
        h, _ = cfm.linear_silu(xn, P[o + 2], P[o + 3], p, s)
        return cfm.linear(h, P[o + 4], P[o + 5], x, p, s + 1, 0.5, f32)

    def mha(x, s):
        xn, _, _ = cfm.layer_norm(x, P[6], P[7], _EPS, cd)
        qkv = cfm.linear(xn, P[8], P[9], None, 0.0, 0, 1.0, cd)
        if layer.pos_enc == "rel":
            pos = cfm.linear(_rel_table(T, d, x.device, cd), R[0], None, None, 0.0, 0, 1.0, cd)
            o, _ = cfm.attention_rel(qkv, pos, R[1].reshape(-1), R[2].reshape(-1), lens, B, T, H, p, s)
        else:
            o, _ = cfm.attention(qkv, lens, B, T, H, p, s)
        return cfm.linear(o, P[10], P[11], x, p, s + 1, 1.0, f32)

    def conv(x, s):
        bn = layer.conv_module.sequential[3]
        xn, _, _ = cfm.layer_norm(x, P[12], P[13], _EPS, cd)
        a = cfm.linear(xn, P[14].view(2 * d, d), P[15], None, 0.0, 0, 1.0, cd)
        train = layer.training or not bn.track_running_stats
        z, _, mean, invstd = cfm.conv_glu_dwconv_bn_silu(
            a, P[16].view(d, K), P[17], P[18], P[19], None if train else bn.running_mean,
            None if train else bn.running_var, train, bn.eps, B, cd)
        if layer.training and bn.track_running_stats:
            m = bn.momentum if bn.momentum is not None else 0.1
            n = B * T
            with torch.no_grad():
                var = (invstd.pow(-2) - bn.eps) * (n / max(n - 1, 1))
                bn.running_mean.mul_(1 - m).add_(mean, alpha=m)
                bn.running_var.mul_(1 - m).add_(var, alpha=m)
        return cfm.linear(z, P[20].view(d, d), P[21], x, p, s, 1.0, f32)

    x1 = ffn(x, 0, seed)
    if layer.convolution_first:
        x3 = mha(conv(x1, seed + 10), seed + 20)
    else:
        x3 = conv(mha(x1, seed + 20), seed + 10)
    x4 = ffn(x3, 22, seed + 30)
    return cfm.layer_norm(x4, P[28], P[29], _EPS, f32)[0]
