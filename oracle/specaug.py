"""Oracle: SpecAugment restated from the reference (TEST INFRASTRUCTURE ONLY).

Reference: /root/reference/lib/standard/asrnn.py
  time_warping       :91-125   per-utterance warp table Wt, then x_warp[b,f,t] = x[b,f,Wt[b,t]]
  frequency_masking  :127-144  draws f, f0 once per call; the mask assignment at :141 writes
                               into a temporary list copy, so the applied mask is all-False
  time_masking       :146-168  draws t, t0 per utterance; :165 likewise never marks the mask
  SpecAugment        :170-192  warping_ntimes warps, frequency_mask_ntimes freq masks, Mt time
                               masks (Mt = min(Mt, floor(pm)) under adaptive_multiplicity)

The random draws use Python's ``random`` module exactly in the reference's order, so the
draw trace (and therefore every mask index) is bit-identical to the reference for the same
seed.  ``apply`` supports mode='reference' (masks are no-ops, as shipped) and
mode='intended' (the masks the code meant to apply).
"""
from __future__ import annotations

import random as _random
from dataclasses import dataclass, field
from math import floor

import numpy as np


@dataclass
class SpecAugDraws:
    """Every random draw one SpecAugment call consumes, in reference order."""
    warps: list = field(default_factory=list)   # per warp pass: list of (w, w0) per utterance
    freq: list = field(default_factory=list)    # per freq-mask pass: (f, f0)
    time: list = field(default_factory=list)    # per time-mask pass: list of (t, t0) per utterance


def draw(n_utts, n_bins, tau, hp, rng=_random):
    """Consume the reference's random draws (asrnn.py:104-108, :138-139, :158-163, :187-189).

    n_utts = x.shape[0], n_bins = x.shape[1] (= v at asrnn.py:137), tau = per-utterance lengths.
    hp needs warping_param_W, warping_ntimes, frequency_mask_param_F, frequency_mask_ntimes,
    time_multiplicity, adaptive_multiplicity, pm, ps, adaptive_size, time_mask_param_T.
    """
    tau = [int(t) for t in tau]
    W = hp.warping_param_W
    d = SpecAugDraws()
    for _ in range(hp.warping_ntimes):                       # asrnn.py:183
        ws = []
        for u in range(n_utts):                               # asrnn.py:102
            w = rng.randint(-W, W)                            # :104
            if tau[u] < 2 * W:                                # :105
                w0 = W                                        # :106
            else:
                w0 = rng.randint(W, tau[u] - W - 1)           # :108
            ws.append((w, w0))
        d.warps.append(ws)
    for _ in range(hp.frequency_mask_ntimes):                 # asrnn.py:185
        f = rng.randint(0, hp.frequency_mask_param_F)         # :138
        f0 = rng.randint(0, n_bins - hp.frequency_mask_param_F)  # :139
        d.freq.append((f, f0))
    Mt = hp.time_multiplicity                                 # :187
    if hp.adaptive_multiplicity:
        Mt = min(Mt, floor(hp.pm))                            # :189
    for _ in range(Mt):
        ts = []
        for u in range(n_utts):                               # :157
            if u < len(tau) and hp.adaptive_size:
                T = floor(hp.ps * tau[u])                     # :159
            else:
                T = hp.time_mask_param_T                      # :161
            t = rng.randint(0, T)                             # :162
            t0 = rng.randint(0, max(tau[u] - T, tau[u]))      # :163
            ts.append((t, t0))
        d.time.append(ts)
    return d


def warp_table(w, w0, tau_u, n_frames):
    """Wt for one utterance (asrnn.py:109-115).

    t <= w0: int(((w0+w)/w0)*t)  (float64 true division, truncation)
    t >  w0: floor(((tau-1-w0-w)*t + (tau-1)*w) / (tau-1-w0))   (integer floor division)
    t >= tau: identity.
    """
    tau_u = int(tau_u)
    out = []
    for t in range(tau_u):
        if t <= w0:
            wt = int(((w0 + w) / w0) * t)
        else:
            wt = ((tau_u - 1 - w0 - w) * t + (tau_u - 1) * w) // (tau_u - 1 - w0)
        out.append(wt)
    out += list(range(len(out), n_frames))
    return out


def apply(x, tau, draws, mode="reference", mask_value=0.0):
    """Apply the drawn SpecAugment to x (B, F, T) float32 numpy; returns a new array.

    Warp gather: asrnn.py:117-124.  Masks: asrnn.py:143 / :167 (no-ops in mode='reference').
    """
    assert mode in ("reference", "intended")
    x = np.array(x, dtype=np.float32, copy=True)
    B, F, T = x.shape
    for ws in draws.warps:
        Wt = np.array([warp_table(w, w0, tau[u], T) for u, (w, w0) in enumerate(ws)], dtype=np.int64)
        x = np.stack([x[b][:, Wt[b]] for b in range(B)], axis=0)
    if mode == "intended":
        for (f, f0) in draws.freq:
            x[:, f0:f0 + f, :] = mask_value
        for ts in draws.time:
            for u, (t, t0) in enumerate(ts):
                x[u, :, t0:t0 + t] = mask_value
    return x

