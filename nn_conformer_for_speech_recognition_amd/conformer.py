"""Conformer encoder on libcfm — drop-in for ``torchaudio.models.Conformer``.

Reference call sites: lib/standard/asrnn.py:29 (construction) and :214 (forward).  Signature,
return values, error behaviour (even depthwise kernel -> ValueError) and state-dict keys are
torchaudio's, so reference checkpoints (runner.py:48-77) load unchanged:

    conformer_layers.{i}.ffn1.sequential.{0,1,4}.*     LayerNorm, Linear(d,ffn), Linear(ffn,d)
    conformer_layers.{i}.self_attn_layer_norm.*
    conformer_layers.{i}.self_attn.{in_proj_weight,in_proj_bias,out_proj.weight,out_proj.bias}
    conformer_layers.{i}.conv_module.layer_norm.*, conv_module.sequential.{0,2,3,5}.*
    conformer_layers.{i}.ffn2.sequential.{0,1,4}.*,  conformer_layers.{i}.final_layer_norm.*
  (+ self_attn.linear_pos.weight, pos_bias_u, pos_bias_v with pos_enc='rel')

Each ConformerLayer runs as ONE autograd node whose forward/backward are sequences of libcfm
kernels (no PyTorch compute ops).  Each layer's input / output (the residual stream between layers) and the
gradient stream are fp32; inside a layer the residual stream is fp32 too (bf16 with the opt-in RES_BF16); GEMM
operands and saved activations use the compute dtype (bf16 by default, fp32 for the parity mode).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from . import ops
from .debug import check as _chk
from ._lib import ACT_SILU

_EPS = 1e-5


class _MHAParams(nn.Module):
    """Parameter holder with nn.MultiheadAttention's names (+ rel-pos extras)."""

    def __init__(self, d, H, dropout, pos_enc):
        super().__init__()
        self.embed_dim, self.num_heads, self.dropout, self.pos_enc = d, H, dropout, pos_enc
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d, bias=True)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)
        if pos_enc == "rel":
            self.linear_pos = nn.Linear(d, d, bias=False)
            self.pos_bias_u = nn.Parameter(torch.empty(H, d // H))
            self.pos_bias_v = nn.Parameter(torch.empty(H, d // H))
            nn.init.xavier_uniform_(self.pos_bias_u)
            nn.init.xavier_uniform_(self.pos_bias_v)


class _FFNParams(nn.Module):
    def __init__(self, d, ffn, dropout):
        super().__init__()
        self.sequential = nn.Sequential(nn.LayerNorm(d), nn.Linear(d, ffn), nn.SiLU(), nn.Dropout(dropout),
                                        nn.Linear(ffn, d), nn.Dropout(dropout))


class _ConvParams(nn.Module):
    def __init__(self, d, K, dropout, use_group_norm):
        super().__init__()
        self.layer_norm = nn.LayerNorm(d)
        self.sequential = nn.Sequential(
            nn.Conv1d(d, 2 * d, 1, bias=True), nn.GLU(dim=1),
            nn.Conv1d(d, d, K, padding=(K - 1) // 2, groups=d, bias=True),
            nn.GroupNorm(1, d) if use_group_norm else nn.BatchNorm1d(d), nn.SiLU(),
            nn.Conv1d(d, d, 1, bias=True), nn.Dropout(dropout))


def rel_pos_table(T, d, device):
    """(2T-1, d) sinusoid, row r <-> relative position (T-1)-r (transformers
    modeling_wav2vec2_conformer.py:168-205).  Built on the host once per length (cached)."""
    pos = torch.arange(T - 1, -T, -1, dtype=torch.int64).float().unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.int64).float() * -(math.log(10000.0) / d))
    pe = torch.zeros(2 * T - 1, d)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.to(device)


# parameter order of one layer (the autograd node's inputs after x)
_PNAMES = [
    "ffn1.sequential.0.weight", "ffn1.sequential.0.bias", "ffn1.sequential.1.weight", "ffn1.sequential.1.bias",
    "ffn1.sequential.4.weight", "ffn1.sequential.4.bias",
    "self_attn_layer_norm.weight", "self_attn_layer_norm.bias",
    "self_attn.in_proj_weight", "self_attn.in_proj_bias", "self_attn.out_proj.weight", "self_attn.out_proj.bias",
    "conv_module.layer_norm.weight", "conv_module.layer_norm.bias",
    "conv_module.sequential.0.weight", "conv_module.sequential.0.bias",
    "conv_module.sequential.2.weight", "conv_module.sequential.2.bias",
    "conv_module.sequential.3.weight", "conv_module.sequential.3.bias",
    "conv_module.sequential.5.weight", "conv_module.sequential.5.bias",
    "ffn2.sequential.0.weight", "ffn2.sequential.0.bias", "ffn2.sequential.1.weight", "ffn2.sequential.1.bias",
    "ffn2.sequential.4.weight", "ffn2.sequential.4.bias",
    "final_layer_norm.weight", "final_layer_norm.bias",
]
_REL_PNAMES = ["self_attn.linear_pos.weight", "self_attn.pos_bias_u", "self_attn.pos_bias_v"]


# rel-pos: all layers' projected tables from one batched GEMM, dW_pos in the grouped weight-gradient launch
# (CFM_REL_BATCH=0: the per-layer projection and weight-gradient GEMMs, A/B)
REL_BATCH = os.environ.get("CFM_REL_BATCH", "1") != "0"
# CFM_RES_BF16=1 (opt-in, bf16 compute only): the residual stream INSIDE each layer (the four sub-module outputs x1,
# x_mha, x_conv, x4) in bf16, as under torch autocast (bf16 GEMM outputs added in bf16); each layer's input and its
# final-LayerNorm output stay fp32, the gradient stream stays fp32.  Measured (round 6, same box): L15 18.42 -> 18.15 ms,
# L60 31.68 -> 31.37 ms, while the 17-layer bf16 errors grow ~2.5x (y 0.6 -> 1.6 %, dx 0.9 -> 1.7 %, worst gradient
# 1.6 -> 2.9 %; rel T 1498 unchanged at 3.6 %): below the 0.6 ms bar set for it, so the fp32 stream stays the default.
RES_BF16 = os.environ.get("CFM_RES_BF16", "0") == "1"
# CFM_RES_FUSE=1 (opt-in, bf16 compute, fp32 stream): each sub-module's residual GEMM writes its output without the
# residual -- bf16 out_scale * dropout(h W^T + b), 2 B per element -- and the next LayerNorm forms x + delta (fp32, the
# stream the backward reads) and normalises it in one pass (cfm_layernorm_fwd_res), instead of the fp32 residual
# epilogue at the end of the GEMM.  Isolated, the GEMMs drop 6 / 5 us (K 2048 / 512) and the LayerNorm grows 2.8 us;
# in the step (round 6, same box, profiles/r06/misc/res_fuse_ab.txt) the GEMMs drop only 28.9 -> 25.3 us while the
# LayerNorms grow 8.4 -> 15.5 us: the unfused LayerNorm reads the stream the GEMM has just written from the Infinity
# Cache, the fused one reads the older x.  L15 18.7 -> 19.0 ms, so the epilogue form stays the default.
RES_FUSE = os.environ.get("CFM_RES_FUSE", "0") == "1"


class _Cfg:
    __slots__ = ("B", "T", "d", "H", "ffn", "K", "p", "cd", "training", "conv_first", "rel", "seed",
                 "bn_rm", "bn_rv", "bn_mom", "pe", "shadow", "shadow_t", "group_wgrad", "layer_index",
                 "grad_dest", "flush_here", "on_flushed", "on_routed", "sync_bn", "shadow8", "pos_pre", "rdt", "rfuse")


# the 2-D (and pointwise-conv) weight matrices of _PNAMES: cast to the compute dtype once per step
_WIDX = (2, 4, 8, 10, 14, 20, 24, 26)
# weights of the forward GEMMs that run on fp8 in fp8 mode: FFN up/down (both FFNs), QKV, out-projection
_FP8_W = (2, 4, 8, 10, 24, 26)
# fp8 scaling: MX block scales (default) or per-tensor current scaling (CFM_FP8_SCALING=tensor, A/B)
FP8_MX = os.environ.get("CFM_FP8_SCALING", "mx") != "tensor"


_SIDE_STREAMS = {}


class _Side:
    """Weight-gradient work of one layer's backward (wgrad GEMMs + bias column sums) on a second
    HIP stream, so it overlaps the data-gradient chain on the main stream.  No record_stream():
    outputs are allocated on the main stream before the side launches, inputs are kept referenced
    until join(), and join() makes the main stream wait for every side launch -- so every block the
    side stream touched is only freed / reused in main-stream order after that wait (also under
    HIP-graph capture, where cross-stream record_stream bookkeeping is fragile)."""

    def __init__(self, device):
        self.main = torch.cuda.current_stream(device)
        key = str(device)
        if key not in _SIDE_STREAMS:
            _SIDE_STREAMS[key] = torch.cuda.Stream(device)
        self.side = _SIDE_STREAMS[key]
        self.keep = []
        self.group = None      # ops.WgradGroup when this layer's weight gradients are deferred
        self.dest = None       # {weight index: (dW view, db view)} in a data-parallel gradient bucket
        self.rgroup = None     # ops.ReduceGroup: this layer's small column reductions, deferred likewise
        self.routed = 0        # grouped weight gradients written straight into their bucket views

    def run(self, fn, *inputs):
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            r = fn()
        self.keep.extend(inputs)
        return r

    def join(self):
        self.main.wait_stream(self.side)
        self.keep = []


# weight gradients of the encoder deferred to ONE grouped launch at the end of its backward (per device),
# and the small column reductions (LayerNorm dgamma|dbeta, depthwise conv dw|db) to one more
_WGRAD_GROUPS = {}
_RED_GROUPS = {}


def _has_grad_hooks(p):
    """True when p has tensor backward hooks or post-accumulate-grad hooks (DDP's reducer, a per-layer
    all-reduce hook, user hooks): those read .grad as soon as AccumulateGrad runs, so the layer's weight
    gradients must not be deferred to the grouped launch.  torch DDP must not wrap this model (it hooks
    every parameter and would disable the grouping); use dist.GradAllReducer."""
    return bool(getattr(p, "_backward_hooks", None)) or bool(getattr(p, "_post_accumulate_grad_hooks", None))


def _wgrad_bias(side, dy, x, widx=None):
    """(dW, db) = (dyᵀ·x, Σ_rows dy): queued for the grouped launch (side.group) when the layer defers its
    weight gradients, else on the side stream (outputs allocated on the main stream).  widx: _PNAMES index
    of the weight; with a data-parallel gradient bucket attached (side.dest, dist.GradAllReducer) the
    grouped launch writes straight into the bucket (autograd adopts the returned views as .grad)."""
    if side.group is not None and ops.wgrad_group_ok(dy, x):
        dest = side.dest.get(widx) if (side.dest and widx is not None) else None
        if dest is not None:
            side.routed += 1
        return side.group.add(dy, x, dest)
    dw = torch.empty(dy.shape[1], x.shape[1], device=dy.device, dtype=torch.float32)
    db = torch.empty(dy.shape[1], device=dy.device, dtype=torch.float32)
    side.run(lambda: ops.linear_wgrad(dy, x, out=dw, bias_out=db), dy, x, dw, db)
    return dw, db


def _w(t, cd):
    """Compute-dtype view of a weight (2-D)."""
    return t if t.dtype == cd else ops.cast(t, cd)


def _wt(cfg, i):
    """K-major (transposed) compute-dtype copy of weight matrix i, if the shadows carry one."""
    return cfg.shadow_t.get(i) if cfg.shadow_t else None


def _fp8_on(cfg, i, K):
    return bool(cfg.shadow8) and i in cfg.shadow8 and K % 128 == 0


def _ln_fwd(x, P, i, cfg, fp8_w=None, d=None):
    """the module-input LayerNorm; when the consumer GEMM (weight fp8_w) runs on MX fp8, the same kernel also
    writes the MX copy of its bf16 output (cfm_layernorm_fwd_mx).  d: the previous module's pending output (RES_FUSE)
    -- the module input is then x + d, formed here.  -> (xn, (xn8, s8) or None, mu, rs, module input)"""
    mx = fp8_w is not None and FP8_MX and cfg.cd == torch.bfloat16 and _fp8_on(cfg, fp8_w, x.shape[1])
    if d is not None:
        if mx:
            x, xn, q, mu, rs = ops.layernorm_fwd_res(x, d, P[i], P[i + 1], _EPS, mx=True)
            return xn, q, mu, rs, x
        x, xn, mu, rs = ops.layernorm_fwd_res(x, d, P[i], P[i + 1], _EPS, out_dtype=cfg.cd)
        return xn, None, mu, rs, x
    if mx:
        xn, q, mu, rs = ops.layernorm_fwd_mx(x, P[i], P[i + 1], _EPS)
        return xn, q, mu, rs, x
    xn, mu, rs = ops.layernorm_fwd(x, P[i], P[i + 1], _EPS, out_dtype=cfg.cd)
    return xn, None, mu, rs, x


def _res_kw(cfg, x):
    """the residual GEMM's output arguments: the new stream (x + ...) or, under RES_FUSE, the bf16 module output"""
    return {"out_dtype": torch.bfloat16} if cfg.rfuse else {"out_dtype": cfg.rdt, "residual": x}


def _fp8_linear(x, cfg, i, xq=None, **kw):
    """Forward GEMM with fp8 (e4m3fn) operands when the layer runs the fp8 path (BASELINE.json configs[4]):
    x quantised on the device -- MX block scales (one e8m0 per 32 K-elements, one pass, applied inside the
    block-scaled MFMA), or per tensor with CFM_FP8_SCALING=tensor (A/B) -- weight i from the per-step fp8 shadow;
    else None.  The backward keeps the bf16 operands (x, the bf16 weight shadow)."""
    if not _fp8_on(cfg, i, x.shape[1]):
        return None
    wq, sw = cfg.shadow8[i]
    if FP8_MX:
        x8, sx = xq if xq is not None else ops.quant_mx(x)
        return ops.linear(x8, wq, x_mx=sx, w_mx=sw, **kw)
    xq, sx = ops.quant_fp8(x)
    return ops.linear(xq, wq, x_scale=sx, w_scale=sw, **kw)


def _ffn_fwd(x, P, o, cfg, seed, d=None):
    """-> (the new stream, or the bf16 module output under RES_FUSE; saved tensors; the module input)"""
    cd = cfg.cd
    xn, xq, mu, rs, x = _ln_fwd(x, P, o, cfg, o + 2, d)
    w1, w2 = _w(P[o + 2], cd), _w(P[o + 4], cd)
    pre = torch.empty(x.shape[0], cfg.ffn, device=x.device, dtype=cd)
    # MX fp8 for both FFN GEMMs: the up-projection's epilogue also writes the MX copy of h (the down GEMM's operand)
    hq = None
    if FP8_MX and _fp8_on(cfg, o + 2, xn.shape[1]) and _fp8_on(cfg, o + 4, cfg.ffn) and cfg.ffn % 32 == 0:
        hq = (torch.empty(x.shape[0], cfg.ffn, device=x.device, dtype=torch.float8_e4m3fn),
              torch.empty(x.shape[0], cfg.ffn // 32, device=x.device, dtype=torch.uint8))
    h = _fp8_linear(xn, cfg, o + 2, xq=xq, bias=P[o + 3], act=ACT_SILU, pre=pre, drop_p=cfg.p, seed=seed,
                    **({"mx_out": hq} if hq is not None else {}))
    if h is None:
        h = ops.linear(xn, w1, P[o + 3], act=ACT_SILU, pre=pre, drop_p=cfg.p, seed=seed)
    y = _fp8_linear(h, cfg, o + 4, xq=hq, bias=P[o + 5], drop_p=cfg.p, seed=seed + 1, out_scale=0.5,
                    **_res_kw(cfg, x))
    if y is None:
        y = ops.linear(h, w2, P[o + 5], drop_p=cfg.p, seed=seed + 1, out_scale=0.5, **_res_kw(cfg, x))
    _chk(f"ffn{o}_fwd", xn, mu, rs, pre, h, y)
    return y, (xn, mu, rs, pre, h, w1, w2), x


def _in_drop(kind, cfg, seed):
    """(scale, p, seed, dtype) of a module's residual-dropout input gradient g2 = scale * mask * g
    (FFN: 0.5 macaron scale; the mask seeds are the forward's)."""
    return {"ffn": (0.5, cfg.p, seed + 1), "mha": (1.0, cfg.p, seed + 1), "conv": (1.0, cfg.p, seed)}[kind] + (cfg.cd,)


def _g2(g, g2, kind, cfg, seed):
    if g2 is not None:
        return g2
    sc, p, sd, cd = _in_drop(kind, cfg, seed)
    return ops.scale_dropout(g, sc, p, sd, 0, out_dtype=cd)


def _ln_bwd(dxn, x, P, i, mu, rs, g, side, nxt):
    """module-input LayerNorm backward (+ residual g); nxt: the next module's _in_drop (or None) ->
    its g2 comes out of the same kernel.  Returns (dx, g2_next)."""
    if nxt is None:
        dx, gg, gb = ops.layernorm_bwd(dxn, x, P[i], mu, rs, dres=g, side=side)
        g2n = None
    else:
        dx, gg, gb, g2n = ops.layernorm_bwd(dxn, x, P[i], mu, rs, dres=g, side=side, drop=nxt)
    return dx, gg, gb, g2n


def _ffn_bwd(g, x, sv, P, o, cfg, seed, grads, side, g2=None, nxt=None):
    xn, mu, rs, pre, h, w1, w2 = sv
    cd = cfg.cd
    g2 = _g2(g, g2, "ffn", cfg, seed)
    grads[o + 4], grads[o + 5] = _wgrad_bias(side, g2, h, o + 4)
    da = ops.linear_dgrad(g2, w2, pre=pre, act_grad=True, drop_p=cfg.p, seed=seed, wt=_wt(cfg, o + 4))
    grads[o + 2], grads[o + 3] = _wgrad_bias(side, da, xn, o + 2)
    dxn = ops.linear_dgrad(da, w1, wt=_wt(cfg, o + 2))
    dx, grads[o], grads[o + 1], g2n = _ln_bwd(dxn, x, P, o, mu, rs, g, side, nxt)
    _chk(f"ffn{o}_bwd", g2, da, dxn, dx, g2n)
    return dx, g2n


def _mha_fwd(x, P, R, cfg, seed, lens, dprev=None):
    cd = cfg.cd
    B, T, d, H = cfg.B, cfg.T, cfg.d, cfg.H
    xn, xq, mu, rs, x = _ln_fwd(x, P, 6, cfg, 8, dprev)
    win, wout = _w(P[8], cd), _w(P[10], cd)
    qkv = _fp8_linear(xn, cfg, 8, xq=xq, bias=P[9])
    if qkv is None:
        qkv = ops.linear(xn, win, P[9])
    pos = pu = pv = None
    if cfg.rel:
        if cfg.pos_pre is not None:     # this layer's slice of Conformer._rel_tables' one batched projection
            pos = cfg.pos_pre
        else:
            pos = ops.linear(_w(cfg.pe, cd), _w(R[0], cd))      # (2T-1, d) projected table (no bias)
        pu = R[1].reshape(-1).float().contiguous()
        pv = R[2].reshape(-1).float().contiguous()
    o, lse = ops.attn_fwd(qkv, lens, B, T, H, d // H, pos, pu, pv, drop_p=cfg.p, seed=seed)
    y = _fp8_linear(o, cfg, 10, bias=P[11], drop_p=cfg.p, seed=seed + 1, **_res_kw(cfg, x))
    if y is None:
        y = ops.linear(o, wout, P[11], drop_p=cfg.p, seed=seed + 1, **_res_kw(cfg, x))
    _chk("mha_fwd", xn, mu, rs, qkv, pos, o, lse, y)
    return y, (xn, mu, rs, qkv, o, lse, win, wout, pos, pu, pv), x


def _mha_bwd(g, x, sv, P, R, cfg, seed, lens, grads, rgrads, side, g2=None, nxt=None):
    xn, mu, rs, qkv, o, lse, win, wout, pos, pu, pv = sv
    cd = cfg.cd
    B, T, d, H = cfg.B, cfg.T, cfg.d, cfg.H
    g4 = _g2(g, g2, "mha", cfg, seed)
    grads[10], grads[11] = _wgrad_bias(side, g4, o, 10)
    wt = _wt(cfg, 10)
    aws = None
    if wt is not None and d // H == 64 and cd == torch.bfloat16 and "rowdot" not in ops.DISABLED:
        # D = rowsum(dO * O) per head from the epilogue of the GEMM producing dO (no separate pass); rel-pos: written
        # into the head of the attention backward's workspace
        # (the full workspace in both cases: the non-rel whole-head path keeps the dS^T its dQ pass reads there)
        aws, Dh = ops.attn_ws(B, T, H, d // H, cfg.rel, g4.device)
        do = ops.linear_dgrad(g4, wout, wt=wt, rowdot=(o, Dh, T))
    else:
        Dh = None
        do = ops.linear_dgrad(g4, wout, wt=wt)
    # rel-pos in bf16: dpos comes back in the compute dtype (the dW_pos GEMM operand; no fp32 copy + cast)
    dpos_dt = torch.bfloat16 if (cfg.rel and cd == torch.bfloat16) else torch.float32
    dqkv, dpos, dpu, dpv = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, d // H, pos, pu, pv, drop_p=cfg.p, seed=seed,
                                        D=Dh, ws=aws, dpos_dtype=dpos_dt)
    if cfg.rel:
        dpc, pec = _w(dpos, cd), _w(cfg.pe, cd)
        if REL_BATCH and side.group is not None and ops.wgrad_group_ok(dpc, pec):
            # dW_pos = dposᵀ·pe as one more task of the grouped weight-gradient launch (M = 2T-1 rows; its bias
            # sums are not used) -- alone it ran on 16 workgroups (L60: 30 us per layer)
            rgrads[0], _ = side.group.add(dpc, pec)
        else:
            rgrads[0] = ops.linear_wgrad(dpc, pec)
        rgrads[1] = dpu.view(H, d // H)
        rgrads[2] = dpv.view(H, d // H)
    grads[8], grads[9] = _wgrad_bias(side, dqkv, xn, 8)
    dxn = ops.linear_dgrad(dqkv, win, wt=_wt(cfg, 8))
    dx, grads[6], grads[7], g2n = _ln_bwd(dxn, x, P, 6, mu, rs, g, side, nxt)
    _chk("mha_bwd", g4, do, Dh, dqkv, dpos, dxn, dx, g2n)
    return dx, g2n


def _conv_fwd(x, P, cfg, seed, dprev=None):
    cd = cfg.cd
    B, T, d, K = cfg.B, cfg.T, cfg.d, cfg.K
    xn, _, mu, rs, x = _ln_fwd(x, P, 12, cfg, None, dprev)
    wp1, wp2 = _w(P[14].view(2 * d, d), cd), _w(P[20].view(d, d), cd)
    wdw = P[16].view(d, K)
    a = ops.linear(xn, wp1, P[15])
    ws = ops.convmod_ws(B, T, d, K, x.device)
    yv = ops.glu_dwconv_fwd(a, wdw, P[17], B, T, d, K, ws)
    if cfg.sync_bn is not None and cfg.training:
        z, bmean, binv = ops.bn_silu_fwd_sync(yv, P[18], P[19], cfg.bn_rm, cfg.bn_rv, cfg.bn_mom, _EPS, B, T, d, ws,
                                              cd, cfg.sync_bn[0], cfg.sync_bn[1])
    else:
        z, bmean, binv = ops.bn_silu_fwd(yv, P[18], P[19], cfg.bn_rm, cfg.bn_rv, cfg.bn_mom, _EPS, cfg.training, B,
                                         T, d, ws, cd)
    y = ops.linear(z, wp2, P[21], drop_p=cfg.p, seed=seed, **_res_kw(cfg, x))
    _chk("conv_fwd", xn, mu, rs, a, yv, bmean, binv, z, y)
    return y, (xn, mu, rs, a, yv, z, bmean, binv, wp1, wp2, wdw), x


def _conv_bwd(g, x, sv, P, cfg, seed, grads, side, g2=None, nxt=None):
    xn, mu, rs, a, yv, z, bmean, binv, wp1, wp2, wdw = sv
    cd = cfg.cd
    B, T, d, K = cfg.B, cfg.T, cfg.d, cfg.K
    g3 = _g2(g, g2, "conv", cfg, seed)
    dw, grads[21] = _wgrad_bias(side, g3, z, 20)
    grads[20] = dw.view(d, d, 1)
    dz = ops.linear_dgrad(g3, wp2, wt=_wt(cfg, 20))
    ws = ops.convmod_ws(B, T, d, K, x.device)
    sync = cfg.sync_bn is not None and cfg.training
    dy = None
    if K in ops.BN_FOLD_K and "bnfold" not in ops.DISABLED:     # (CFM_DISABLE=bnfold: separate BN backward, A/B)
        da, dwdw, grads[17], grads[18], grads[19] = ops.bn_silu_glu_dwconv_bwd(
            dz, yv, P[18], P[19], bmean, binv, cfg.training, a, wdw, B, T, d, K, ws, cd, side=side,
            reduce_sums=cfg.sync_bn[0] if sync else None, world=cfg.sync_bn[1] if sync else 1)
    else:
        if sync:
            dy, grads[18], grads[19] = ops.bn_silu_bwd_sync(dz, yv, P[18], P[19], bmean, binv, ws, cfg.sync_bn[0],
                                                            cfg.sync_bn[1])
        else:
            dy, grads[18], grads[19] = ops.bn_silu_bwd(dz, yv, P[18], P[19], bmean, binv, cfg.training, ws)
        da, dwdw, grads[17] = ops.glu_dwconv_bwd(dy, a, wdw, B, T, d, K, ws, cd, side=side)
    grads[16] = dwdw.view(d, 1, K)
    dw, grads[15] = _wgrad_bias(side, da, xn, 14)
    grads[14] = dw.view(2 * d, d, 1)
    dxn = ops.linear_dgrad(da, wp1, wt=_wt(cfg, 14))
    dx, grads[12], grads[13], g2n = _ln_bwd(dxn, x, P, 12, mu, rs, g, side, nxt)
    _chk("conv_bwd", g3, dz, dy, grads[18], grads[19], da, dxn, dx, g2n)
    return dx, g2n


class _ConformerLayerFn(torch.autograd.Function):
    """One torchaudio ConformerLayer as a single autograd node over libcfm."""

    @staticmethod
    def forward(ctx, x, lens, cfg, *params):
        P = list(params[:len(_PNAMES)])
        R = params[len(_PNAMES):]
        if cfg.shadow is not None:       # compute-dtype copies refreshed by Conformer (one launch)
            for i, t in cfg.shadow[0].items():
                P[i] = t
            cfg.shadow_t = cfg.shadow[1]
            cfg.shadow8 = cfg.shadow[2] if len(cfg.shadow) > 2 else None
        else:
            cfg.shadow_t = cfg.shadow8 = None
        s = cfg.seed
        x0 = x
        # each module returns its output (the new stream; under RES_FUSE the pending bf16 module output, added by the
        # next LayerNorm) and its input, materialised by that LayerNorm -- the tensors the backward saves
        y1, sv1, _ = _ffn_fwd(x0, P, 0, cfg, s)
        step = (lambda xin, y: (xin, y)) if cfg.rfuse else (lambda xin, y: (y, None))
        cur = step(x0, y1)
        if cfg.conv_first:
            yc, svc, x1 = _conv_fwd(cur[0], P, cfg, s + 10, cur[1])
            cur = step(x1, yc)
            ya, sva, xc = _mha_fwd(cur[0], P, R, cfg, s + 20, lens, cur[1])
            cur = step(xc, ya)
            chain = (x1, xc)
        else:
            ya, sva, x1 = _mha_fwd(cur[0], P, R, cfg, s + 20, lens, cur[1])
            cur = step(x1, ya)
            yc, svc, xa = _conv_fwd(cur[0], P, cfg, s + 10, cur[1])
            cur = step(xa, yc)
            chain = (x1, xa)
        y4, sv4, x3 = _ffn_fwd(cur[0], P, 22, cfg, s + 30, cur[1])
        cur = step(x3, y4)
        if cur[1] is not None:
            x4, out, mu5, rs5 = ops.layernorm_fwd_res(cur[0], cur[1], P[28], P[29], _EPS, out_dtype=torch.float32)
        else:
            x4 = cur[0]
            out, mu5, rs5 = ops.layernorm_fwd(x4, P[28], P[29], _EPS, out_dtype=torch.float32)
        _chk(f"layer{cfg.layer_index}_fwd_out", out, mu5, rs5)
        ctx.cfg = cfg
        ctx.sv = (sv1, sva, svc, sv4)
        ctx.save_for_backward(x0, chain[0], chain[1], x3, x4, mu5, rs5, lens, *params)
        return out

    @staticmethod
    def backward(ctx, gout):
        cfg = ctx.cfg
        saved = ctx.saved_tensors
        x0, c0, c1, x3, x4, mu5, rs5, lens = saved[:8]
        params = saved[8:]
        P = params[:len(_PNAMES)]
        R = params[len(_PNAMES):]
        sv1, sva, svc, sv4 = ctx.sv
        grads = [None] * len(_PNAMES)
        rgrads = [None] * len(R)
        s = cfg.seed
        gout = gout.contiguous()
        side = _Side(gout.device)
        # defer this layer's weight-gradient GEMMs into the encoder-wide grouped launch (flushed by layer 0,
        # the last to run backward) when no parameter accumulates into an existing .grad
        # (never when a parameter carries a gradient hook: hooks fire as .grad lands, before the flush)
        if cfg.group_wgrad and all(p.grad is None and not _has_grad_hooks(p) for p in params):
            side.group = _WGRAD_GROUPS.setdefault(str(gout.device), ops.WgradGroup())
            side.group.arm_final_flush()
            side.dest = cfg.grad_dest
            if "rgroup" not in ops.DISABLED:     # (CFM_DISABLE=rgroup: per-layer side-stream reductions, A/B)
                side.rgroup = _RED_GROUPS.setdefault(str(gout.device), ops.ReduceGroup())
                side.rgroup.arm_final_flush()
        # each LayerNorm backward also emits the next module's dropout-scaled input gradient (g2)
        ffn2_in = _in_drop("ffn", cfg, s + 30)
        conv_in, mha_in, ffn1_in = _in_drop("conv", cfg, s + 10), _in_drop("mha", cfg, s + 20), _in_drop("ffn", cfg, s)
        if "lndrop" in ops.DISABLED:
            ffn2_in = conv_in = mha_in = ffn1_in = None
        if ffn2_in is None:
            (g, grads[28], grads[29]), g2 = ops.layernorm_bwd(gout, x4, P[28], mu5, rs5, side=side), None
        else:
            g, grads[28], grads[29], g2 = ops.layernorm_bwd(gout, x4, P[28], mu5, rs5, side=side, drop=ffn2_in)
        if cfg.conv_first:
            g, g2 = _ffn_bwd(g, x3, sv4, P, 22, cfg, s + 30, grads, side, g2, mha_in)
            g, g2 = _mha_bwd(g, c1, sva, P, R, cfg, s + 20, lens, grads, rgrads, side, g2, conv_in)
            g, g2 = _conv_bwd(g, c0, svc, P, cfg, s + 10, grads, side, g2, ffn1_in)
        else:
            g, g2 = _ffn_bwd(g, x3, sv4, P, 22, cfg, s + 30, grads, side, g2, conv_in)
            g, g2 = _conv_bwd(g, c1, svc, P, cfg, s + 10, grads, side, g2, mha_in)
            g, g2 = _mha_bwd(g, c0, sva, P, R, cfg, s + 20, lens, grads, rgrads, side, g2, ffn1_in)
        g, _ = _ffn_bwd(g, x0, sv1, P, 0, cfg, s, grads, side, g2, None)
        side.join()
        if cfg.on_routed is not None and side.dest and side.routed == len(side.dest):
            cfg.on_routed(cfg.layer_index)       # (data-parallel reducer: this layer's buckets are final at flush)
        if cfg.layer_index == 0 or cfg.flush_here:
            # layer 0 runs backward last: everything deferred is flushed; data-parallel runs also flush at
            # bucket boundaries so the bucket's all-reduce (on_flushed) overlaps the remaining backward
            grp = _WGRAD_GROUPS.get(str(gout.device))
            if grp is not None:
                grp.flush()
            rgrp = _RED_GROUPS.get(str(gout.device))
            if rgrp is not None:
                rgrp.flush()
            if cfg.on_flushed is not None:
                cfg.on_flushed(cfg.layer_index)
        _chk(f"layer{cfg.layer_index}_bwd_dx", g)
        ctx.sv = None
        return (g, None, None, *grads, *rgrads)


class ConformerLayer(nn.Module):
    """torchaudio.models.conformer.ConformerLayer (parameter names and semantics)."""

    def __init__(self, input_dim, ffn_dim, num_attention_heads, depthwise_conv_kernel_size, dropout=0.0,
                 use_group_norm=False, convolution_first=False, pos_enc="none"):
        super().__init__()
        if use_group_norm:
            raise NotImplementedError("use_group_norm=True: GroupNorm conv module is not on the MI355X path yet")
        self.ffn1 = _FFNParams(input_dim, ffn_dim, dropout)
        self.self_attn_layer_norm = nn.LayerNorm(input_dim)
        self.self_attn = _MHAParams(input_dim, num_attention_heads, dropout, pos_enc)
        self.self_attn_dropout = nn.Dropout(dropout)
        self.conv_module = _ConvParams(input_dim, depthwise_conv_kernel_size, dropout, use_group_norm)
        self.ffn2 = _FFNParams(input_dim, ffn_dim, dropout)
        self.final_layer_norm = nn.LayerNorm(input_dim)
        self.convolution_first = convolution_first
        self.dropout = dropout
        self.pos_enc = pos_enc
        self.d, self.H, self.ffn, self.K = input_dim, num_attention_heads, ffn_dim, depthwise_conv_kernel_size

    def params(self):
        sd = dict(self.named_parameters())
        ps = [sd[n] for n in _PNAMES]
        if self.pos_enc == "rel":
            ps += [sd[n] for n in _REL_PNAMES]
        return ps

    def forward_tokens(self, x, lens_i32, B, T, compute_dtype, seed, pe=None, shadow=None, layer_index=0,
                       group_wgrad=False, grad_dest=None, flush_here=False, on_flushed=None, sync_bn=None,
                       count_batches=True, on_routed=None, pos_pre=None):
        """x: (B*T, d) fp32 token-major; lens_i32: (B,) int32 on the device; shadow: optional
        ({param index: compute-dtype copy}, {param index: its transposed K-major copy}) of this
        layer's weight matrices (see Conformer._shadows)."""
        cfg = _Cfg()
        cfg.shadow = shadow
        cfg.B, cfg.T, cfg.d, cfg.H, cfg.ffn, cfg.K = B, T, self.d, self.H, self.ffn, self.K
        cfg.p = float(self.dropout) if self.training else 0.0
        cfg.cd = compute_dtype
        cfg.rdt = torch.bfloat16 if (compute_dtype == torch.bfloat16 and RES_BF16) else torch.float32
        cfg.rfuse = compute_dtype == torch.bfloat16 and RES_FUSE and not RES_BF16
        cfg.training = self.training
        cfg.conv_first = self.convolution_first
        cfg.rel = self.pos_enc == "rel"
        cfg.seed = seed
        bn = self.conv_module.sequential[3]
        cfg.bn_rm, cfg.bn_rv = bn.running_mean, bn.running_var
        cfg.bn_mom = bn.momentum if bn.momentum is not None else 0.1
        cfg.pe = pe
        cfg.pos_pre = pos_pre
        cfg.layer_index = layer_index
        cfg.group_wgrad = bool(group_wgrad) and "wgroup" not in ops.DISABLED
        cfg.grad_dest, cfg.flush_here, cfg.on_flushed, cfg.on_routed = grad_dest, flush_here, on_flushed, on_routed
        cfg.sync_bn = sync_bn
        if count_batches and self.training and bn.track_running_stats:
            bn.num_batches_tracked.add_(1)
        return _ConformerLayerFn.apply(x, lens_i32, cfg, *self.params())


class Conformer(nn.Module):
    """Drop-in for torchaudio.models.Conformer (asrnn.py:29):
    Conformer(input_dim, num_heads, ffn_dim, num_layers, depthwise_conv_kernel_size, dropout=0.0,
              use_group_norm=False, convolution_first=False)
    plus build knobs pos_enc ('none' | 'rel') and compute_dtype (torch.bfloat16 | torch.float32).
    forward(input (B, T, D), lengths (B,)) -> (output (B, T, D), lengths)."""

    def __init__(self, input_dim, num_heads, ffn_dim, num_layers, depthwise_conv_kernel_size, dropout=0.0,
                 use_group_norm=False, convolution_first=False, pos_enc="none", compute_dtype=torch.bfloat16,
                 fp8=False):
        super().__init__()
        if depthwise_conv_kernel_size % 2 != 1:
            raise ValueError("depthwise_conv_kernel_size must be odd to achieve 'SAME' padding.")
        if input_dim % num_heads != 0:
            raise ValueError("input_dim must be divisible by num_heads")
        if pos_enc not in ("none", "rel"):
            raise ValueError(f"pos_enc must be 'none' or 'rel', got {pos_enc!r}")
        self.conformer_layers = nn.ModuleList([
            ConformerLayer(input_dim, ffn_dim, num_heads, depthwise_conv_kernel_size, dropout, use_group_norm,
                           convolution_first, pos_enc) for _ in range(num_layers)])
        self.input_dim = input_dim
        self.pos_enc = pos_enc
        self.compute_dtype = compute_dtype
        if fp8 and compute_dtype != torch.bfloat16:
            raise ValueError("fp8=True needs compute_dtype=torch.bfloat16 (the backward runs in bf16)")
        # fp8 (e4m3fn) forward GEMMs (FFN up/down, QKV, out-projection; K % 128 == 0): BASELINE configs[4]
        self.fp8 = bool(fp8)
        self._pe_cache = {}       # (device, dtype) -> (longest T, its (2T-1, d) table): _pe slices it
        self._pe_retired = []     # superseded tables (a captured graph may still read one)
        self._rel_cache = None    # (device, dtype, weight storage) -> linear_pos weight stack + its cast batch
        self._step = 0
        self._shadow = None
        self._q8 = None         # (key, ops.Quant8Batch) of the fp8 forward weights
        # data-parallel hooks (dist.GradAllReducer.attach): per-layer {weight index: (dW, db) bucket views},
        # the layers whose backward flushes the grouped launch, and the callback run after each flush
        self.grad_dest = None
        self.flush_layers = frozenset()
        self.on_flushed = None
        self.on_routed = None
        self.sync_bn = None     # (reduce_sums(t) in-place all-reduce, world) -> cross-replica BatchNorm

    def _pe(self, T, device, dtype=torch.float32):
        """The (2T-1, d) positional table of length T in `dtype`, as the middle rows of ONE table built for the
        longest length seen: row r of the Tcap table is relative position (Tcap-1)-r and its values depend on the
        position alone, so rows Tcap-T .. Tcap+T-2 ARE the length-T table, bit for bit.  Variable-length batches
        therefore share one table per (device, dtype) instead of one per distinct T.  It grows geometrically; a
        superseded table is kept referenced (a captured graph may still read it), so the memory stays below about
        twice the longest table."""
        key = (str(device), dtype)
        ent = self._pe_cache.get(key)
        if ent is None or ent[0] < T:
            tcap = max(T, 2 * ent[0]) if ent is not None else T
            full = rel_pos_table(tcap, self.input_dim, device)
            if dtype != torch.float32:
                full = ops.cast(full, dtype)
            if ent is not None:
                self._pe_retired.append(ent[1])
            ent = (tcap, full)
            self._pe_cache[key] = ent
        tcap, full = ent
        return full[tcap - T:tcap + T - 1]

    def _rel_tables(self, T, device):
        """rel-pos: the compute-dtype positional table (a slice of the shared table, _pe) and every layer's
        projected table pos_l = pe · W_pos,lᵀ from ONE batched GEMM (pe shared, batch = layers) over a per-step
        stacked compute-dtype copy of the linear_pos weights (one cast launch) -- per layer this was a cast of pe, a
        cast of W_pos and a 48-workgroup GEMM (L60: ~24 us per layer).  The weight stack does not depend on T (one
        entry, keyed on the weights' storage); the projected tables are allocated per forward (the backward saves
        them; under graph capture they come from the graph's pool), so no per-length buffers accumulate.
        -> (pe in the compute dtype, (L, 2T-1, d) tables)"""
        cd, d, nl = self.compute_dtype, self.input_dim, len(self.conformer_layers)
        ws = [ly.self_attn.linear_pos.weight for ly in self.conformer_layers]
        key = (str(device), cd, tuple(w.data_ptr() for w in ws))
        if self._rel_cache is None or self._rel_cache[0] != key:
            wstack = torch.empty(nl, d, d, device=device, dtype=cd)
            cb = None if cd == torch.float32 else ops.CastBatch([w.detach() for w in ws], [wstack[i] for i in range(nl)])
            self._rel_cache = (key, wstack, cb)
        _, wstack, cb = self._rel_cache
        if cb is not None:
            cb.refresh()
        else:
            for i, w in enumerate(ws):
                wstack[i].copy_(w.detach())
        pe_cd = self._pe(T, device, cd)
        pos_all = torch.empty(nl, 2 * T - 1, d, device=device, dtype=cd)
        ops.gemm(pe_cd, wstack, pos_all, 2 * T - 1, d, d, batch=nl, stride_a=0, stride_b=d * d,
                 stride_c=(2 * T - 1) * d)
        return pe_cd, pos_all

    def _shadows(self, device):
        """Compute-dtype copies of every layer's weight matrices and their transposes, refreshed by
        ONE cfm_cast_transpose_batch launch per forward (instead of one cast per matrix per layer)."""
        if self.compute_dtype == torch.float32:
            return [None] * len(self.conformer_layers)
        srcs = [layer.params()[i] for layer in self.conformer_layers for i in _WIDX]
        key = (str(device), tuple(t.data_ptr() for t in srcs))
        if self._shadow is None or self._shadow[0] != key:
            n = len(_WIDX)
            dsts = [torch.empty(t.shape, device=device, dtype=self.compute_dtype) for t in srcs]
            # K-major copies Wᵀ (K, N) for the data-gradient GEMMs (pointwise convs viewed 2-D)
            srcs2 = [t.detach().view(t.shape[0], -1) for t in srcs]   # detached: no autograd view nodes kept alive
            dsts_t = [torch.empty(t.shape[1], t.shape[0], device=device, dtype=self.compute_dtype) for t in srcs2]
            per = [(dict(zip(_WIDX, dsts[j * n:(j + 1) * n])), dict(zip(_WIDX, dsts_t[j * n:(j + 1) * n])))
                   for j in range(len(self.conformer_layers))]
            self._shadow = (key, ops.CastTBatch(srcs2, dsts_t, dsts), per)   # one launch, one read
        self._shadow[1].refresh()
        if not self.fp8:
            return self._shadow[2]
        # per-step fp8 copies (+ dequantisation scalars) of the forward GEMM weights, from the fp32 masters: ONE
        # batched quantisation (two launches for all layers; was two launches per weight)
        if getattr(self, "_q8", None) is None or self._q8[0] != key:
            srcs8 = [layer.params()[i].detach().view(layer.params()[i].shape[0], -1)
                     for layer in self.conformer_layers for i in _FP8_W]
            self._q8 = (key, ops.QuantMXBatch(srcs8) if FP8_MX else ops.Quant8Batch(srcs8))
        outs = self._q8[1].refresh()
        nw = len(_FP8_W)
        out = []
        for j, (plain, trans) in enumerate(self._shadow[2]):
            q8 = dict(zip(_FP8_W, outs[j * nw:(j + 1) * nw]))
            out.append((plain, trans, q8))
        return out

    def set_sync_batchnorm(self, group=None):
        """torch.nn.SyncBatchNorm semantics for every ConvModule BatchNorm (train mode): batch statistics and
        the input-gradient sums over all replicas of `group` (default: the default process group), one
        all-reduce of 2*d floats per BN per pass; each rank's weight/bias gradients stay local (the data-
        parallel gradient all-reduce averages them).  group=False turns it off."""
        import torch.distributed as dist
        if group is False or not (dist.is_available() and dist.is_initialized()):
            self.sync_bn = None
            return self
        world = dist.get_world_size(group)
        self.sync_bn = (lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group), world)
        return self

    def forward_tokens(self, x, lens_i32, B, T, seed=None):
        if torch.compiler.is_compiling():
            return self._forward_tokens_ops(x, lens_i32, B, T, seed)
        if seed is None:
            seed = (self._step * 1000003 + 12345) & 0x7FFFFFFF
            self._step += 1
        pe = pos_all = None
        if self.pos_enc == "rel":
            if REL_BATCH:
                pe, pos_all = self._rel_tables(T, x.device)
            else:
                pe = self._pe(T, x.device)
        shadows = self._shadows(x.device)
        # grouped weight gradients need layer 0 to run backward last (it flushes the group): true for the
        # sequential encoder; deferral is per layer and falls back when a .grad accumulates
        group = self.compute_dtype == torch.bfloat16
        for i, layer in enumerate(self.conformer_layers):
            x = layer.forward_tokens(x, lens_i32, B, T, self.compute_dtype, seed + 100 * i, pe, shadows[i],
                                     layer_index=i, group_wgrad=group,
                                     grad_dest=self.grad_dest[i] if self.grad_dest else None,
                                     flush_here=i in self.flush_layers, on_flushed=self.on_flushed,
                                     sync_bn=self.sync_bn, count_batches=False, on_routed=self.on_routed,
                                     pos_pre=None if pos_all is None else pos_all[i])
        # every layer's BatchNorm num_batches_tracked += 1 in one multi-tensor launch (not one per layer)
        counters = [ly.conv_module.sequential[3].num_batches_tracked for ly in self.conformer_layers
                    if self.training and ly.conv_module.sequential[3].track_running_stats]
        if counters:
            torch._foreach_add_(counters, 1)
        return x

    def _forward_tokens_ops(self, x, lens_i32, B, T, seed):
        """The encoder as torch.ops.cfm.* calls (library.layer_forward): the route torch.compile traces
        (fullgraph=True).  Same kernels as the fused layer node; dropout seeds are fixed per call site unless
        `seed` is given (a device step counter bound with cfm_rng_bind salts them per step, as in HIP-graph
        replay), so no Python-side step counter is mutated inside the traced region.
        The guard below sees only THAT a counter is bound, not that it advances: the caller owns advancing it once
        per step, outside the compiled region (bench.py's Harness adds 1 to its counter before every replay); a
        bound but frozen counter replays the same masks every step."""
        from . import library, _lib
        if seed is None and self.training and not _lib.RNG_BOUND and any(
                float(ly.dropout) > 0 for ly in self.conformer_layers):
            # fixed per-call-site seeds would apply the SAME dropout masks every compiled step
            raise RuntimeError("compiled Conformer training with dropout > 0 needs fresh masks per step: pass "
                               "seed=<per-step int> to forward_tokens or bind a device step counter "
                               "(cfm_rng_bind) whose value advances every step")
        base = 12345 if seed is None else seed
        for i, layer in enumerate(self.conformer_layers):
            x = library.layer_forward(layer, x, lens_i32, B, T, self.compute_dtype, base + 100 * i)
        for ly in self.conformer_layers:
            bn = ly.conv_module.sequential[3]
            if self.training and bn.track_running_stats:
                bn.num_batches_tracked.add_(1)
        return x

    def forward(self, input, lengths):
        if input.dim() != 3 or input.shape[-1] != self.input_dim:
            raise ValueError(f"expected input (B, T, {self.input_dim}), got {tuple(input.shape)}")
        if not input.is_cuda:
            raise RuntimeError("Conformer runs on libcfm HIP kernels: move the module and inputs to the GPU")
        B, T, d = input.shape
        lens = lengths.to(device=input.device, dtype=torch.int32)
        x = input.reshape(B * T, d).float().contiguous()
        y = self.forward_tokens(x, lens, B, T)
        return y.view(B, T, d).to(input.dtype), lengths
