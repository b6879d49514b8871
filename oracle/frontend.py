"""Oracle: convolution front-end and encoder glue (TEST INFRASTRUCTURE ONLY), torch CPU fp32.

ConvSubSampling   /root/reference/lib/convsubsampling.py:16-45
    Conv2d(in→C1, k1, stride s1) → Conv2d(C1→C2, k2, stride s2); no activation, no padding;
    out_size = C2·H'·W' with H' = (H-k+s)//s per stage (:26-32).
standard_linear   /root/reference/lib/standard/asrnn.py:28,207-209 — whole-utterance Linear
    (out_size → d·max_len), view (B, max_len, d).  ('utterance' projection)
frame projection  SURVEY.md §8a A8 — permute (B,C2,F',T') → (B,T',C2·F') and Linear(C2·F', d).
encoder           asrnn.py:193-221 — SpecAugment? → convsub → projection → dropout →
    crop to non-zero lengths and max length → Conformer → pad back → flatten → projection_block
    (Linear → SiLU → BatchNorm1d, asrnn.py:73-89).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def stage_len(n, k, s):
    """(n - k + s) // s — convsubsampling.py:30-31."""
    return (n - k + s) // s


def convsub_forward(x, w1, b1, w2, b2, s1=(2, 2), s2=(2, 2)):
    """x (B, 1, F, T) → (B, C2, F', T') (convsubsampling.py:43-45)."""
    return F.conv2d(F.conv2d(x, w1, b1, stride=s1), w2, b2, stride=s2)


def frame_projection(y, w, b):
    """y (B, C2, F', T') → (B, T', d): per-subsampled-frame Linear over the frame's (f', c2)
    features (feature index f'*C2 + c2 — the build's 'frame' projection)."""
    B, C2, Fp, Tp = y.shape
    feats = y.permute(0, 3, 2, 1).reshape(B, Tp, Fp * C2)
    return F.linear(feats, w, b)


def utterance_projection(y, w, b, max_len):
    """asrnn.py:207-209: flatten(1) → Linear(out_size, d·max_len) → view(B, max_len, d)."""
    B = y.shape[0]
    z = F.linear(y.flatten(1), w, b)
    return z.view(B, max_len, z.shape[1] // max_len)


def frame_lengths(tau, k1=7, s1=2, k2=3, s2=2):
    """Subsampled valid-frame count per utterance (same arithmetic as convsubsampling.py:30-31)."""
    return stage_len(stage_len(tau, k1, s1), k2, s2)
