"""CPU: the CTC oracle (oracle/ctc.py) pinned against torch.nn.functional.ctc_loss on the CPU —
the reference's own loss call (runner.py:35,142-143: CTCLoss(blank, zero_infinity=True) on
log_softmax outputs) — loss and logits gradient, incl. repeated labels, empty targets, padded
frames and infeasible (infinite, zeroed) utterances; and the greedy-decode filter."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ctc as oc


def _case(seed, B=4, T=12, V=7, S=4):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, T, V, generator=g, dtype=torch.float64) * 2
    tgt = torch.randint(1, V, (B, S), generator=g)
    tgt[0, 1] = tgt[0, 0]                       # repeated label (needs a blank between)
    il = torch.tensor([T, T - 3, T, 2][:B])     # last: 2 frames for 3 labels -> infeasible
    tl = torch.tensor([S, 2, 0, 3][:B])         # incl. an empty target
    return x, tgt, il, tl


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_matches_torch_ctc(seed, reduction):
    x, tgt, il, tl = _case(seed)
    xr = x.clone().requires_grad_()
    lp = F.log_softmax(xr, -1).transpose(0, 1)
    ref = F.ctc_loss(lp, tgt, il, tl, blank=0, reduction=reduction, zero_infinity=True)
    (ref.sum() if reduction == "none" else ref).backward()
    loss, grad = oc.ctc_loss(x.numpy(), tgt.numpy(), il.numpy(), tl.numpy(), 0, reduction, True)
    np.testing.assert_allclose(np.asarray(loss), ref.detach().numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(grad, xr.grad.numpy(), rtol=1e-8, atol=1e-10)


def test_oracle_blank_not_zero():
    x, tgt, il, tl = _case(3, V=6)
    tgt = torch.where(tgt == 5, torch.ones_like(tgt), tgt)     # labels avoid blank=5
    xr = x.clone().requires_grad_()
    ref = F.ctc_loss(F.log_softmax(xr, -1).transpose(0, 1), tgt, il, tl, blank=5, zero_infinity=True)
    ref.backward()
    loss, grad = oc.ctc_loss(x.numpy(), tgt.numpy(), il.numpy(), tl.numpy(), 5, "mean", True)
    np.testing.assert_allclose(loss, ref.item(), rtol=1e-10)
    np.testing.assert_allclose(grad, xr.grad.numpy(), rtol=1e-8, atol=1e-10)


def test_oracle_greedy_filter():
    logits = np.zeros((2, 6, 4))
    seq = [[0, 2, 2, 0, 3, 1], [1, 1, 0, 0, 2, 3]]
    for b in range(2):
        for t, c in enumerate(seq[b]):
            logits[b, t, c] = 1.0
    ids, out = oc.greedy_decode(logits, blank=0, pad=1)
    assert ids.tolist() == seq
    assert out == [[2, 2, 3], [2, 3]]                 # reference: no repeat collapse
    _, out_c = oc.greedy_decode(logits, lens=[6, 4], blank=0, pad=-1, collapse=True)
    assert out_c == [[2, 3, 1], [1]]
