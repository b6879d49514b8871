"""Oracle: torchaudio Conformer semantics (+ Transformer-XL rel-pos MHSA), torch CPU fp32.

TEST INFRASTRUCTURE ONLY.

The reference builds ``torchaudio.models.Conformer(input_dim=512, num_heads=8, ffn_dim=512,
num_layers=1, depthwise_conv_kernel_size=33, dropout=0.5)`` at
/root/reference/lib/standard/asrnn.py:29 and calls it at :214.  torchaudio is not vendored and
not installed here, so this module restates its semantics:

  padding_mask = arange(max(lengths)) >= lengths[:, None]        (key padding only)
  per layer:  x += 0.5*FFN1(x);  x += MHSA(LN(x));  x += Conv(x);  x += 0.5*FFN2(x);  x = LN(x)
  FFN  = LN → Linear(d,ffn) → SiLU → Dropout → Linear(ffn,d) → Dropout
  Conv = LN → Conv1d(d,2d,1) → GLU(dim=1) → depthwise Conv1d(d,K,pad (K-1)//2) → BatchNorm1d
         → SiLU → Conv1d(d,d,1) → Dropout          (padded frames are NOT zeroed)
  MHSA = nn.MultiheadAttention(d, H, dropout) with packed in_proj, key_padding_mask

Relative positions (pos_enc='rel') follow transformers' Wav2Vec2ConformerSelfAttention
(modeling_wav2vec2_conformer.py:159-205, :528-565): pe has 2T-1 rows for relative positions
+(T-1)..-(T-1) (sin in even, cos in odd columns), p = linear_pos(pe) (no bias),
scores = ((q+u)·kᵀ + (q+v)·p[(T-1)-(i-j)]ᵀ) / sqrt(dk).

Module and parameter names are torchaudio's so state dicts are interchangeable with the
product's ``Conformer`` (and with checkpoints the reference saves, runner.py:48-77).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def rel_pos_table(T, d, dtype=torch.float32):
    """(2T-1, d) sinusoid table, row r ↔ relative position (T-1)-r (HF :168-205)."""
    pos = torch.arange(T - 1, -T, -1, dtype=torch.int64).float().unsqueeze(1)   # +(T-1) .. -(T-1)
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.int64).float() * -(math.log(10000.0) / d))
    pe = torch.zeros(2 * T - 1, d)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.to(dtype)


class FeedForwardRef(nn.Module):
    """torchaudio _FeedForwardModule (names: sequential.{0,1,4})."""

    def __init__(self, d, ffn, dropout=0.0):
        super().__init__()
        self.sequential = nn.Sequential(nn.LayerNorm(d), nn.Linear(d, ffn, bias=True), nn.SiLU(),
                                        nn.Dropout(dropout), nn.Linear(ffn, d, bias=True), nn.Dropout(dropout))

    def forward(self, x):
        return self.sequential(x)


class ConvModuleRef(nn.Module):
    """torchaudio _ConvolutionModule (names: layer_norm, sequential.{0,2,3,5})."""

    def __init__(self, d, K, dropout=0.0, use_group_norm=False):
        super().__init__()
        if (K - 1) % 2 != 0:
            raise ValueError("depthwise_kernel_size must be odd to achieve 'SAME' padding.")
        self.layer_norm = nn.LayerNorm(d)
        self.sequential = nn.Sequential(
            nn.Conv1d(d, 2 * d, 1, stride=1, padding=0, bias=True),
            nn.GLU(dim=1),
            nn.Conv1d(d, d, K, stride=1, padding=(K - 1) // 2, groups=d, bias=True),
            nn.GroupNorm(num_groups=1, num_channels=d) if use_group_norm else nn.BatchNorm1d(d),
            nn.SiLU(),
            nn.Conv1d(d, d, 1, stride=1, padding=0, bias=True),
            nn.Dropout(dropout),
        )

    def forward(self, x):           # x (B, T, d)
        y = self.layer_norm(x).transpose(1, 2)
        return self.sequential(y).transpose(1, 2)


class RelPosMHARef(nn.Module):
    """nn.MultiheadAttention-named parameters plus linear_pos / pos_bias_u / pos_bias_v."""

    def __init__(self, d, H, dropout=0.0, pos_enc="none"):
        super().__init__()
        self.d, self.H, self.dk = d, H, d // H
        self.dropout = dropout
        self.pos_enc = pos_enc
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d, bias=True)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)
        if pos_enc == "rel":
            self.linear_pos = nn.Linear(d, d, bias=False)
            self.pos_bias_u = nn.Parameter(torch.zeros(H, self.dk))
            self.pos_bias_v = nn.Parameter(torch.zeros(H, self.dk))
            nn.init.xavier_uniform_(self.pos_bias_u)
            nn.init.xavier_uniform_(self.pos_bias_v)

    def forward(self, x, key_padding_mask):          # x (B, T, d); mask (B, T) True = pad
        B, T, d = x.shape
        H, dk = self.H, self.dk
        qkv = F.linear(x, self.in_proj_weight, self.in_proj_bias)
        q, k, v = qkv.split(d, dim=-1)
        q = q.view(B, T, H, dk).transpose(1, 2)
        k = k.view(B, T, H, dk).transpose(1, 2)
        v = v.view(B, T, H, dk).transpose(1, 2)
        if self.pos_enc == "rel":
            pe = rel_pos_table(T, d, x.dtype)
            p = self.linear_pos(pe).view(2 * T - 1, H, dk).transpose(0, 1)       # (H, 2T-1, dk)
            ac = torch.matmul(q + self.pos_bias_u[None, :, None, :], k.transpose(-2, -1))
            bd_full = torch.matmul(q + self.pos_bias_v[None, :, None, :], p.transpose(-2, -1)[None])
            i = torch.arange(T)[:, None]
            j = torch.arange(T)[None, :]
            idx = (T - 1) - i + j                                                  # (T, T)
            bd = torch.gather(bd_full, 3, idx[None, None].expand(B, H, T, T))
            scores = (ac + bd) / math.sqrt(dk)
        else:
            scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(dk)
        scores = scores.masked_fill(key_padding_mask[:, None, None, :], float("-inf"))
        probs = torch.softmax(scores, dim=-1)
        if self.training and self.dropout > 0:
            probs = F.dropout(probs, self.dropout)
        o = torch.matmul(probs, v).transpose(1, 2).reshape(B, T, d)
        return self.out_proj(o)


class ConformerLayerRef(nn.Module):
    """torchaudio ConformerLayer (names: ffn1, self_attn_layer_norm, self_attn, self_attn_dropout,
    conv_module, ffn2, final_layer_norm)."""

    def __init__(self, d, ffn, H, K, dropout=0.0, use_group_norm=False, convolution_first=False,
                 pos_enc="none"):
        super().__init__()
        self.ffn1 = FeedForwardRef(d, ffn, dropout)
        self.self_attn_layer_norm = nn.LayerNorm(d)
        self.self_attn = RelPosMHARef(d, H, dropout, pos_enc)
        self.self_attn_dropout = nn.Dropout(dropout)
        self.conv_module = ConvModuleRef(d, K, dropout, use_group_norm)
        self.ffn2 = FeedForwardRef(d, ffn, dropout)
        self.final_layer_norm = nn.LayerNorm(d)
        self.convolution_first = convolution_first

    def _conv(self, x):
        return x + self.conv_module(x)

    def forward(self, x, key_padding_mask):           # (B, T, d)
        x = x + 0.5 * self.ffn1(x)
        if self.convolution_first:
            x = self._conv(x)
        r = x
        y = self.self_attn(self.self_attn_layer_norm(x), key_padding_mask)
        x = self.self_attn_dropout(y) + r
        if not self.convolution_first:
            x = self._conv(x)
        x = x + 0.5 * self.ffn2(x)
        return self.final_layer_norm(x)


def lengths_to_padding_mask(lengths, T=None):
    T = int(lengths.max().item()) if T is None else T
    return torch.arange(T, device=lengths.device)[None, :] >= lengths[:, None]


class ConformerRef(nn.Module):
    """torchaudio.models.Conformer signature (asrnn.py:29): (input_dim, num_heads, ffn_dim,
    num_layers, depthwise_conv_kernel_size, dropout, use_group_norm, convolution_first)."""

    def __init__(self, input_dim, num_heads, ffn_dim, num_layers, depthwise_conv_kernel_size,
                 dropout=0.0, use_group_norm=False, convolution_first=False, pos_enc="none"):
        super().__init__()
        self.conformer_layers = nn.ModuleList([
            ConformerLayerRef(input_dim, ffn_dim, num_heads, depthwise_conv_kernel_size, dropout,
                              use_group_norm, convolution_first, pos_enc)
            for _ in range(num_layers)])

    def forward(self, input, lengths):                # (B, T, d), (B,)
        mask = lengths_to_padding_mask(lengths, input.shape[1])
        x = input
        for layer in self.conformer_layers:
            x = layer(x, mask)
        return x, lengths


def seeded_hf_compatible(d, H, ffn, L, K, pos_enc, seed):
    """Deterministic Conformer weights for the golden fixtures (test infrastructure): torch.manual_seed(seed)
    init, then non-trivial biases / LayerNorm / BatchNorm affine params, conv-module conv biases zeroed
    (transformers' Wav2Vec2Conformer conv module has none).  The CPU generator makes this reproducible on
    any machine, so big fixtures store the seed instead of the weights."""
    torch.manual_seed(seed)
    ref = ConformerRef(d, H, ffn, L, K, 0.0, pos_enc=pos_enc)
    with torch.no_grad():
        for layer in ref.conformer_layers:
            for m in (layer.conv_module.sequential[0], layer.conv_module.sequential[2],
                      layer.conv_module.sequential[5]):
                m.bias.zero_()
            for nm, p in layer.named_parameters():
                if nm.endswith("bias") and "conv_module.sequential" not in nm:
                    p.normal_(0, 0.1)
                if "layer_norm" in nm and nm.endswith("weight"):
                    p.uniform_(0.5, 1.5)
            layer.conv_module.sequential[3].weight.uniform_(0.5, 1.5)
            layer.conv_module.sequential[3].bias.normal_(0, 0.1)
    return ref


def grad_probes(name, g, k=16):
    """k fixed random projections of a (large) gradient tensor -- the compact fixture form of a weight
    gradient: probes[i] = <R_i, g> with R_i ~ N(0, 1) from a generator seeded by the parameter name."""
    gen = torch.Generator().manual_seed(sum(ord(c) * (i + 1) for i, c in enumerate(name)) % (2 ** 31))
    R = torch.randn(k, g.numel(), generator=gen, dtype=torch.float64)
    return R @ g.reshape(-1).double()
