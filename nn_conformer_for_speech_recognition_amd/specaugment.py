"""SpecAugment (ASRNN.SpecAugment, lib/standard/asrnn.py:170-192) on the GPU.

Host side: the random draws use python ``random`` — the reference's own RNG, which the dataset
seeds at import (speechcommands.py:18) — in exactly the reference's order, so every warp and
mask index is bit-identical to the reference for the same seed.  For data-parallel training
the draws are made for the GLOBAL batch and each rank applies its slice (``rank_slice``).

Device side: one HIP kernel (cfm_specaug_apply) composes the warp gathers and applies the masks
in a single HBM pass — no per-frame Python loop, no device→host round trip (asrnn.py:113,117).
"""
from __future__ import annotations

import random as _random
from math import floor

import torch

from . import _lib as L


def draw(n_utts, n_bins, tau, hp, rng=_random):
    """Return (warps, freqs, times) drawn in the order of asrnn.py:183-191.

    warps: per warp pass, [(w, w0)] per utterance     (time_warping :104-108)
    freqs: per freq-mask pass, (f, f0)                 (frequency_masking :138-139)
    times: per time-mask pass, [(t, t0)] per utterance (time_masking :158-163)
    Raises ValueError exactly where the reference's randint would (e.g. tau = 2W).
    """
    W = hp.warping_param_W
    tau = [int(t) for t in tau]
    warps, freqs, times = [], [], []
    for _ in range(hp.warping_ntimes):
        per = []
        for u in range(n_utts):
            w = rng.randint(-W, W)
            w0 = W if tau[u] < 2 * W else rng.randint(W, tau[u] - W - 1)
            per.append((w, w0))
        warps.append(per)
    for _ in range(hp.frequency_mask_ntimes):
        f = rng.randint(0, hp.frequency_mask_param_F)
        freqs.append((f, rng.randint(0, n_bins - hp.frequency_mask_param_F)))
    n_time = hp.time_multiplicity
    if hp.adaptive_multiplicity:
        n_time = min(n_time, floor(hp.pm))
    for _ in range(n_time):
        per = []
        for u in range(n_utts):
            T = floor(hp.ps * tau[u]) if (u < len(tau) and hp.adaptive_size) else hp.time_mask_param_T
            t = rng.randint(0, T)
            per.append((t, rng.randint(0, max(tau[u] - T, tau[u]))))
        times.append(per)
    return warps, freqs, times


def pack(draws, tau, lo=0, hi=None):
    """int32 parameter block of cfm_specaug_apply for utterances [lo, hi) of the drawn batch."""
    warps, freqs, times = draws
    n = len(warps[0]) if warps else (len(times[0]) if times else len(tau))
    hi = n if hi is None else hi
    out = [len(warps), len(freqs), len(times), 0]
    for per in warps:
        for u in range(lo, hi):
            w, w0 = per[u]
            out += [w, w0, int(tau[u])]
    for f, f0 in freqs:
        out += [f0, f]
    for per in times:
        for u in range(lo, hi):
            t, t0 = per[u]
            out += [t0, t]
    return torch.tensor(out, dtype=torch.int32)


def apply(x, params_dev, intended, mask_value=0.0):
    """x (B, F, T) fp32 device tensor → augmented copy (one kernel)."""
    if x.dim() != 3 or x.dtype != torch.float32:
        raise ValueError("SpecAugment expects (B, F, T) float32")
    B, F, T = x.shape
    y = torch.empty_like(x)
    L.call("cfm_specaug_apply", L.ptr(x), L.ptr(y), B, F, T, L.ptr(params_dev), params_dev.numel(),
           int(bool(intended)), float(mask_value), L.stream())
    return y


def spec_augment(x, tau, hp, intended=None, rng=_random, rank_slice=None):
    """Draw + apply.  x: (B, F, T) or (B, 1, F, T) on the GPU; tau: lengths (list or tensor).

    intended=None follows hp.specaug_ref_noop_masks (True → the reference's no-op masks).
    rank_slice=(lo, hi): x holds utterances [lo, hi) of a global batch of len(tau) utterances.
    """
    squeeze = x.dim() == 4
    xs = x.reshape(x.shape[0], x.shape[-2], x.shape[-1]) if squeeze else x
    tau_l = [int(t) for t in (tau.tolist() if torch.is_tensor(tau) else tau)]
    n_glob = len(tau_l) if rank_slice is not None else xs.shape[0]
    for t in tau_l:
        if t > xs.shape[-1]:
            raise ValueError(f"utterance length {t} exceeds the frame count {xs.shape[-1]}")
    draws = draw(n_glob, xs.shape[1], tau_l, hp, rng)
    lo, hi = rank_slice if rank_slice is not None else (0, xs.shape[0])
    params = pack(draws, tau_l, lo, hi).to(x.device, non_blocking=True)
    if intended is None:
        intended = not getattr(hp, "specaug_ref_noop_masks", False)
    y = apply(xs.contiguous(), params, intended, float(getattr(hp, "mask_value", 0)))
    return y.reshape(x.shape) if squeeze else y
