"""Oracle: CTC head of the training step and greedy decode (TEST INFRASTRUCTURE ONLY), numpy fp64.

The reference's loss is torch.nn.CTCLoss(blank=hp.blank_idx, zero_infinity=True) built at
/root/reference/lib/standard/runner.py:35 and applied at runner.py:142-143 to the log-softmax
output of ASRNN.forward (asrnn.py:45,256); its decode is ASRNN.predict (asrnn.py:48-58:
torch.argmax) followed by Vocab.decode's filter (myvocab.py:211-231: drop <pad>/<blank>, no
repeat collapse).  This module restates torch's published CTC algorithm (Graves et al. 2006
alpha/beta in log space; torch's LossCTC conventions: beta includes the emission at t, the
gradient is taken w.r.t. the logits through log_softmax, 'mean' divides by max(target length, 1)
before the batch mean, zero_infinity zeroes infinite losses and their gradients) in plain loops.
It is pinned against torch.nn.functional.ctc_loss on the CPU — the reference's own call — by
tests/test_ctc_oracle.py.  Only tests/ may import it.
"""
from __future__ import annotations

import numpy as np


def _lse(*v):
    m = max(v)
    if m == -np.inf:
        return -np.inf
    return m + np.log(sum(np.exp(x - m) for x in v))


def log_softmax(x):
    m = x.max(-1, keepdims=True)
    return x - m - np.log(np.exp(x - m).sum(-1, keepdims=True))


def ctc_utterance(lp, tgt, blank):
    """lp (T, V) log-probs of one utterance (frames < input length), tgt (L,) labels.
    Returns (nll, grad_logits (T, V)) with grad = softmax - posterior (unscaled)."""
    T, V = lp.shape
    ext = [blank]
    for c in tgt:
        ext += [int(c), blank]
    S = len(ext)
    if T == 0:
        return (0.0 if len(tgt) == 0 else np.inf), np.zeros((0, V))
    alpha = np.full((T, S), -np.inf)
    beta = np.full((T, S), -np.inf)
    alpha[0, 0] = lp[0, ext[0]]
    if S > 1:
        alpha[0, 1] = lp[0, ext[1]]
    for t in range(1, T):
        for s in range(S):
            terms = [alpha[t - 1, s]]
            if s >= 1:
                terms.append(alpha[t - 1, s - 1])
            if s >= 2 and ext[s] != blank and ext[s] != ext[s - 2]:
                terms.append(alpha[t - 1, s - 2])
            alpha[t, s] = _lse(*terms) + lp[t, ext[s]]
    beta[T - 1, S - 1] = lp[T - 1, ext[S - 1]]
    if S > 1:
        beta[T - 1, S - 2] = lp[T - 1, ext[S - 2]]
    for t in range(T - 2, -1, -1):
        for s in range(S):
            terms = [beta[t + 1, s]]
            if s + 1 < S:
                terms.append(beta[t + 1, s + 1])
            if s + 2 < S and ext[s] != blank and ext[s] != ext[s + 2]:
                terms.append(beta[t + 1, s + 2])
            beta[t, s] = _lse(*terms) + lp[t, ext[s]]
    nll = -_lse(alpha[T - 1, S - 1], alpha[T - 1, S - 2] if S > 1 else -np.inf)
    grad = np.exp(lp).copy()
    if np.isfinite(nll):
        for t in range(T):
            for s in range(S):
                grad[t, ext[s]] -= np.exp(alpha[t, s] + beta[t, s] + nll - lp[t, ext[s]])
    return nll, grad


def ctc_loss(logits, targets, in_len, tgt_len, blank=0, reduction="mean", zero_infinity=True):
    """logits (B, T, V) (log_softmax is applied, as the reference's model does), targets (B, S) padded.
    Returns (loss, grad_logits (B, T, V)) for grad_out = 1."""
    logits = np.asarray(logits, dtype=np.float64)
    B, T, V = logits.shape
    lp = log_softmax(logits)
    nll = np.zeros(B)
    grads = np.zeros_like(logits)
    for b in range(B):
        n, g = ctc_utterance(lp[b, :in_len[b]], targets[b, :tgt_len[b]], blank)
        if zero_infinity and np.isinf(n):
            n, g = 0.0, np.zeros_like(g)
        nll[b] = n
        grads[b, :in_len[b]] = g
    if reduction == "none":
        return nll, grads
    if reduction == "sum":
        return nll.sum(), grads
    w = 1.0 / (B * np.maximum(np.asarray(tgt_len, dtype=np.float64), 1.0))
    return float((nll * w).sum()), grads * w[:, None, None]


def greedy_decode(logits, lens=None, blank=0, pad=-1, collapse=False):
    """argmax ids (B, T) and the filtered per-utterance id lists (asrnn.py:48-58, myvocab.py:225-228)."""
    ids = np.asarray(logits).argmax(-1)
    out = []
    for b in range(ids.shape[0]):
        n = ids.shape[1] if lens is None else int(lens[b])
        seq, prev = [], None
        for t in range(n):
            c = int(ids[b, t])
            rep = collapse and c == prev
            prev = c
            if rep or c == blank or c == pad:
                continue
            seq.append(c)
        out.append(seq)
    return ids, out
