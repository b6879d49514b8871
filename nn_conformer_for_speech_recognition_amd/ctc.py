"""CTC head on libcfm — drop-ins for the reference's loss and decode calls.

  CTCLoss / ctc_loss   torch.nn.CTCLoss(blank=hp.blank_idx, zero_infinity=True) as built at
                       runner.py:35 and applied at runner.py:142-143 to the log-probabilities of
                       ASRNN.forward (asrnn.py:256).  Same arguments, layouts ((T, B, V) by default),
                       reductions and zero_infinity behaviour; log_softmax is fused (idempotent on
                       log-probabilities), so raw logits may be passed too.
  ctc_head_loss        the fused head of the training step: Linear(d -> V) + log_softmax + CTC as ONE
                       autograd node (no fp32 logits gradient round trip: the CTC kernel writes the
                       logits gradient in the compute dtype straight into the head's two GEMMs).
  greedy_decode        ASRNN.predict (asrnn.py:48-58, argmax) + the id filter of Vocab.decode
                       (myvocab.py:211-231: <pad>/<blank> dropped, no repeat collapse by default).

Everything is stream-ordered with no host synchronisation when targets are padded (B, S) and the
lengths are device tensors, so a whole training step can be captured into one HIP graph.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops

_RED = ("none", "mean", "sum")


def _lengths(v, B, device, limit=None, what="lengths"):
    """(B,) int32 device lengths.  Host-side lengths (lists, CPU tensors) are validated against
    `limit` as torch.nn.functional.ctc_loss does (it raises); device lengths are not read back (no
    sync) -- the kernels clamp them to the buffers' extents instead."""
    if isinstance(v, (list, tuple)):
        v = torch.tensor(v)
    if not torch.is_tensor(v):
        raise TypeError("lengths must be tensors or sequences of ints")
    if v.numel() != B:
        raise ValueError(f"expected {B} lengths, got {v.numel()}")
    if not v.is_cuda and v.numel() > 0:
        lo, hi = int(v.min()), int(v.max())
        if lo < 0:
            raise ValueError(f"{what} must be non-negative, got {lo}")
        if limit is not None and hi > limit:
            raise ValueError(f"expected {what} to have value at most {limit}, but got value {hi}")
    return v.to(device=device, dtype=torch.int32).contiguous()


def _check_blank(blank, V):
    if not 0 <= blank < V:
        raise ValueError(f"blank must be in label range [0, {V}), got {blank}")


def _prep_targets(targets, tgt_len, B, device):
    """(targets int32, ldt, offsets or None, Smax) for padded (B, S) or concatenated 1-D targets."""
    if targets.dim() == 2:
        t = targets.to(device=device, dtype=torch.int32).contiguous()
        return t, t.shape[1], None, t.shape[1]
    if targets.dim() == 1:
        t = targets.to(device=device, dtype=torch.int32).contiguous()
        off = (torch.cumsum(tgt_len, 0, dtype=torch.int32) - tgt_len).contiguous()
        smax = int(tgt_len.max().item()) if B > 0 else 0     # host sync (1-D form only)
        return t, 0, off, smax
    raise ValueError("targets must be (B, S) padded or 1-D concatenated")


_NONFINITE = None


def set_nonfinite_counter(counter):
    """Bind a (1,) int32 device counter that every reduction='mean' CTC loss increments when its value is not
    finite (no host sync; e.g. a training loop's bad-step count, read once after the run).  None unbinds."""
    global _NONFINITE
    if counter is not None and (counter.dtype != torch.int32 or counter.numel() != 1 or not counter.is_cuda):
        raise ValueError("nonfinite counter: a (1,) int32 CUDA tensor")
    _NONFINITE = counter


def _reduce(nll, tl, reduction):
    if reduction == "none":
        return nll
    if reduction == "sum":
        return nll.sum()
    # mean_b(nll_b / max(L_b, 1)) as one launch (cfm_ctc_mean; was clamp + cast + divide + mean)
    return ops.ctc_mean(nll, tl, _NONFINITE)


class _CTCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, in_len, tgt_len, blank, reduction, zero_infinity, batch_first):
        if not x.is_cuda or x.dtype != torch.float32:
            raise RuntimeError("ctc_loss runs on libcfm: fp32 CUDA log-probs/logits required")
        x = x if x.stride(-1) == 1 else x.contiguous()
        B = x.shape[0] if batch_first else x.shape[1]
        T = x.shape[1] if batch_first else x.shape[0]
        _check_blank(blank, x.shape[-1])
        il = _lengths(in_len, B, x.device, T, "input_lengths")
        tl = _lengths(tgt_len, B, x.device, targets.shape[1] if targets.dim() == 2 else None, "target_lengths")
        tg, ldt, off, smax = _prep_targets(targets, tl, B, x.device)
        nll, ws = ops.ctc_loss_fwd(x, tg, ldt, off, il, tl, smax, blank, zero_infinity, batch_first)
        ctx.save_for_backward(x, tg, off if off is not None else tg, il, tl, ws)
        ctx.cfg = (ldt, off is not None, smax, blank, zero_infinity, batch_first, reduction)
        return _reduce(nll, tl, reduction)

    @staticmethod
    def backward(ctx, g):
        x, tg, off, il, tl, ws = ctx.saved_tensors
        ldt, has_off, smax, blank, zi, bf, red = ctx.cfg
        dx = ops.ctc_loss_bwd(x, tg, ldt, off if has_off else None, il, tl, smax, blank, zi, bf, ws, g, red)
        return dx, None, None, None, None, None, None, None


def ctc_loss(log_probs, targets, input_lengths, target_lengths, blank=0, reduction="mean", zero_infinity=False,
             batch_first=False):
    """torch.nn.functional.ctc_loss on libcfm (log_probs (T, B, V), or (B, T, V) if batch_first)."""
    if reduction not in _RED:
        raise ValueError(f"{reduction} is not a valid value for reduction")
    return _CTCFn.apply(log_probs, targets, input_lengths, target_lengths, int(blank), reduction,
                        bool(zero_infinity), bool(batch_first))


class CTCLoss(nn.Module):
    """torch.nn.CTCLoss(blank=0, reduction='mean', zero_infinity=False) on libcfm."""

    def __init__(self, blank=0, reduction="mean", zero_infinity=False):
        super().__init__()
        if reduction not in _RED:
            raise ValueError(f"{reduction} is not a valid value for reduction")
        self.blank, self.reduction, self.zero_infinity = blank, reduction, zero_infinity

    def forward(self, log_probs, targets, input_lengths, target_lengths):
        return ctc_loss(log_probs, targets, input_lengths, target_lengths, self.blank, self.reduction,
                        self.zero_infinity)


class _CTCHeadFn(torch.autograd.Function):
    """y (B*T, d) -> logits = y·Wᵀ + b (fp32, batch-major) -> CTC loss; backward writes the logits
    gradient in the compute dtype and runs the head's dgrad / wgrad GEMMs on it directly."""

    @staticmethod
    def forward(ctx, y, w, b, targets, in_len, tgt_len, B, T, blank, reduction, zero_infinity, cd):
        yc = y if y.dtype == cd else ops.cast(y, cd)
        wc = w if w.dtype == cd else ops.cast(w, cd)
        logits = ops.linear(yc, wc, b, out_dtype=torch.float32).view(B, T, -1)
        _check_blank(blank, w.shape[0])
        il = _lengths(in_len, B, y.device, T, "input_lengths")
        tl = _lengths(tgt_len, B, y.device, targets.shape[1] if targets.dim() == 2 else None, "target_lengths")
        tg, ldt, off, smax = _prep_targets(targets, tl, B, y.device)
        nll, ws = ops.ctc_loss_fwd(logits, tg, ldt, off, il, tl, smax, blank, zero_infinity, True)
        ctx.save_for_backward(logits, yc, wc, tg, off if off is not None else tg, il, tl, ws)
        ctx.cfg = (ldt, off is not None, smax, blank, zero_infinity, reduction, cd, y.dtype, b is not None)
        ctx.mark_non_differentiable(logits)
        ctx.set_materialize_grads(False)     # no (B, T, V) zero gradient for the logits output
        return _reduce(nll, tl, reduction), logits

    @staticmethod
    def backward(ctx, g, _glogits):
        logits, yc, wc, tg, off, il, tl, ws = ctx.saved_tensors
        ldt, has_off, smax, blank, zi, red, cd, ydt, has_b = ctx.cfg
        dl = ops.ctc_loss_bwd(logits, tg, ldt, off if has_off else None, il, tl, smax, blank, zi, True, ws, g, red,
                              grad_dtype=cd)
        dl2 = dl.view(-1, dl.shape[-1])
        dw = ops.linear_wgrad(dl2, yc)
        db = ops.colsum(dl2) if has_b else None
        dy = ops.linear_dgrad(dl2, wc, out_dtype=ydt)
        return dy, dw, db, None, None, None, None, None, None, None, None, None


def ctc_head_loss(y, weight, bias, targets, input_lengths, target_lengths, B, T, blank=0, reduction="mean",
                  zero_infinity=True, compute_dtype=torch.bfloat16):
    """Fused Linear(d -> V) + log_softmax + CTC over token-major encoder rows y (B*T, d).
    Returns (loss, logits (B, T, V) fp32 — e.g. for greedy_decode; not differentiable)."""
    if reduction not in _RED:
        raise ValueError(f"{reduction} is not a valid value for reduction")
    return _CTCHeadFn.apply(y, weight, bias, targets, input_lengths, target_lengths, int(B), int(T), int(blank),
                            reduction, bool(zero_infinity), compute_dtype)


def greedy_decode(logits, lengths=None, blank=0, pad=-1, collapse=False, batch_first=True, compact=True):
    """ASRNN.predict + Vocab.decode's id filter on the device.
    Returns (ids (B, T) int64 = torch.argmax(logits, -1), tokens (B, T) int32 padded with -1, n (B,));
    compact=False: ids only (tokens, n are None)."""
    if not logits.is_cuda or logits.dtype != torch.float32:
        raise RuntimeError("greedy_decode runs on libcfm: fp32 CUDA logits required")
    x = logits if logits.stride(-1) == 1 else logits.contiguous()
    B = x.shape[0] if batch_first else x.shape[1]
    ln = None if lengths is None else _lengths(lengths, B, x.device)
    return ops.ctc_greedy_decode(x, ln, blank, pad, collapse, batch_first, compact)
