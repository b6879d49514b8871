"""GPU parity of the CTC head (ctc.hip) against the CPU oracle (oracle/ctc.py, itself pinned to
torch.nn.functional.ctc_loss — the reference's loss call, runner.py:35,142-143) and torch CPU.

Tolerances (fp32 kernels, fp64 references): loss rel 1e-5, logits gradient abs 1e-5 x max|grad|
(fp32 exp/log chains over T frames); fused bf16 head: rel 2e-2 on parameter / input gradients."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from nn_conformer_for_speech_recognition_amd import ctc
from oracle import ctc as oc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(seed, B=4, T=12, V=7, S=4):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, T, V, generator=g) * 2
    tgt = torch.randint(1, V, (B, S), generator=g)
    tgt[0, 1] = tgt[0, 0]
    il = torch.tensor([T, T - 3, T, 2][:B])
    tl = torch.tensor([S, 2, 0, 3][:B])
    return x, tgt, il, tl


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
@pytest.mark.parametrize("batch_first", [False, True])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ctc_loss_vs_oracle(seed, batch_first, reduction):
    x, tgt, il, tl = _case(seed)
    loss_ref, grad_ref = oc.ctc_loss(x.double().numpy(), tgt.numpy(), il.numpy(), tl.numpy(), 0, reduction, True)
    xd = (x if batch_first else x.transpose(0, 1).contiguous()).to(DEV).requires_grad_()
    loss = ctc.ctc_loss(xd, tgt.to(DEV), il.to(DEV), tl.to(DEV), blank=0, reduction=reduction, zero_infinity=True,
                        batch_first=batch_first)
    (loss.sum() if reduction == "none" else loss).backward()
    np.testing.assert_allclose(loss.detach().cpu().double().numpy(), loss_ref, rtol=1e-5, atol=1e-6)
    g = xd.grad.cpu().double()
    g = g if batch_first else g.transpose(0, 1)
    np.testing.assert_allclose(g.numpy(), grad_ref, atol=1e-7 + 1e-5 * np.abs(grad_ref).max())


def test_ctc_module_log_probs_and_concat_targets():
    """torch.nn.CTCLoss drop-in: (T, B, V) log-probabilities, 1-D concatenated targets, blank != 0."""
    x, tgt, il, tl = _case(5, V=9)
    tgt = torch.where(tgt == 8, torch.ones_like(tgt), tgt)
    flat = torch.cat([tgt[b, :tl[b]] for b in range(tgt.shape[0])])
    xr = x.double().clone().requires_grad_()
    lp_ref = F.log_softmax(xr, -1).transpose(0, 1)
    ref = F.ctc_loss(lp_ref, flat, il, tl, blank=8, zero_infinity=True)
    ref.backward()
    lp = F.log_softmax(x.to(DEV), -1).transpose(0, 1).detach().requires_grad_()
    loss = ctc.CTCLoss(blank=8, zero_infinity=True)(lp, flat.to(DEV), il.to(DEV), tl.to(DEV))
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    # gradient w.r.t. the log-probs equals torch's gradient w.r.t. log_probs
    lp64 = F.log_softmax(x.double(), -1).transpose(0, 1).clone().requires_grad_()
    F.ctc_loss(lp64, flat, il, tl, blank=8, zero_infinity=True).backward()
    want = lp64.grad.numpy()
    np.testing.assert_allclose(lp.grad.cpu().double().numpy(), want, atol=1e-7 + 1e-5 * np.abs(want).max())


def test_ctc_bench_shape_vs_torch():
    """The bench workload's head: B=32, T=373 encoder frames, V=1024, U=93 labels, random lengths."""
    g = torch.Generator().manual_seed(7)
    B, T, V, U = 32, 373, 1024, 93
    x = torch.randn(B, T, V, generator=g)
    tgt = torch.randint(1, V, (B, U), generator=g)
    il = torch.randint(T // 2, T + 1, (B,), generator=g)
    il[0] = T
    tl = torch.randint(1, U + 1, (B,), generator=g)
    xr = x.double().clone().requires_grad_()
    ref = F.ctc_loss(F.log_softmax(xr, -1).transpose(0, 1), tgt, il, tl, zero_infinity=True)
    ref.backward()
    xd = x.to(DEV).requires_grad_()
    loss = ctc.ctc_loss(xd, tgt.to(DEV), il.to(DEV), tl.to(DEV), zero_infinity=True, batch_first=True)
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    gd = xd.grad.cpu().double()
    # fp32 log-space recursions over 373 frames lose ~1e-4 absolute in alpha+beta (|log p| ~ 2.6e3),
    # so the posterior carries ~1e-3 relative error in ANY fp32 CTC: hold the kernel to the
    # reference's own fp32 CPU CTC's distance from fp64 (x2), not to fp64 itself
    x32 = x.clone().requires_grad_()
    F.ctc_loss(F.log_softmax(x32, -1).transpose(0, 1), tgt, il, tl, zero_infinity=True).backward()
    err_ref32 = (x32.grad.double() - xr.grad).abs().max().item()
    err = (gd - xr.grad).abs().max().item()
    assert err <= 2 * err_ref32 + 1e-7, (err, err_ref32)
    # every valid frame's gradient sums to zero over classes (softmax - posterior)
    s = gd.sum(-1)
    assert s.abs().max().item() < 1e-3 * xr.grad.abs().max().item()


def test_ctc_head_fused_vs_torch():
    g = torch.Generator().manual_seed(11)
    B, T, d, V, U = 4, 40, 64, 48, 8
    y = torch.randn(B * T, d, generator=g)
    w = torch.randn(V, d, generator=g) * 0.1
    b = torch.randn(V, generator=g) * 0.1
    tgt = torch.randint(1, V, (B, U), generator=g)
    il = torch.tensor([T, T - 5, T, 20])
    tl = torch.tensor([U, 5, 3, U])
    yr, wr, br = (t.clone().requires_grad_() for t in (y, w, b))
    lg = (yr.bfloat16().float() @ wr.bfloat16().float().T + br).view(B, T, V)
    ref = F.ctc_loss(F.log_softmax(lg, -1).transpose(0, 1), tgt, il, tl, zero_infinity=True)
    ref.backward()
    yd, wd, bd = (t.to(DEV).requires_grad_() for t in (y, w, b))
    loss, logits = ctc.ctc_head_loss(yd, wd, bd, tgt.to(DEV), il.to(DEV), tl.to(DEV), B, T, zero_infinity=True)
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 1e-3 * abs(ref.item())
    for got, want in ((yd.grad, yr.grad), (wd.grad, wr.grad), (bd.grad, br.grad)):
        rel = (got.cpu() - want).norm() / want.norm()
        assert rel < 2e-2, rel
    assert logits.shape == (B, T, V)


@pytest.mark.parametrize("collapse", [False, True])
def test_greedy_decode_vs_oracle(collapse):
    g = torch.Generator().manual_seed(3)
    B, T, V = 6, 50, 12
    x = torch.randn(B, T, V, generator=g)
    x[:, ::3, 0] += 3.0                    # plenty of blanks
    x[:, 5:9, :] = x[:, 5:6, :]            # repeats
    lens = torch.tensor([50, 40, 1, 0, 25, 50])
    ids_ref, out_ref = oc.greedy_decode(x.numpy(), lens.numpy(), blank=0, pad=1, collapse=collapse)
    ids, out, n = ctc.greedy_decode(x.to(DEV), lens.to(DEV), blank=0, pad=1, collapse=collapse)
    assert torch.equal(ids.cpu(), torch.argmax(x, -1))
    assert ids.cpu().numpy().tolist() == ids_ref.tolist()
    for b in range(B):
        assert out[b, :n[b]].cpu().tolist() == out_ref[b]
        assert (out[b, n[b]:] == -1).all()


def test_ctc_bad_host_lengths_raise():
    """torch.nn.functional.ctc_loss raises on input_lengths > T / target_lengths > S: so does the
    drop-in when the lengths are host data (lengths are never trusted)."""
    x, tgt, il, tl = _case(3)
    xd = x.to(DEV)
    T, S = x.shape[1], tgt.shape[1]
    with pytest.raises(ValueError):
        ctc.ctc_loss(xd, tgt.to(DEV), torch.tensor([T + 1, 3, 3, 2]), tl, batch_first=True)
    with pytest.raises(ValueError):
        ctc.ctc_loss(xd, tgt.to(DEV), il, torch.tensor([S + 2, 1, 1, 1]), batch_first=True)
    with pytest.raises(ValueError):
        ctc.ctc_loss(xd, tgt.to(DEV), il, tl, blank=x.shape[-1], batch_first=True)


def test_ctc_bad_device_lengths_are_clamped():
    """Device lengths are not read back (no sync): the kernels clamp in_len to T, tgt_len to S and
    label ids to [0, V) -- the result equals the clamped inputs' loss and no memory outside the
    buffers is touched (guard tensors around the workspace stay intact)."""
    x, tgt, il, tl = _case(4)
    B, T, V = x.shape
    S = tgt.shape[1]
    bad_il = torch.tensor([T + 50, T - 3, 10 ** 6, 2], dtype=torch.int32)
    bad_tl = torch.tensor([S + 7, 2, 0, 10 ** 5], dtype=torch.int32)
    bad_tg = tgt.clone()
    bad_tg[1, 0] = V + 3
    guard = torch.full((1 << 16,), 7.0, device=DEV)
    xd = x.to(DEV).requires_grad_()
    loss = ctc.ctc_loss(xd, bad_tg.to(DEV), bad_il.to(DEV), bad_tl.to(DEV), reduction="none", zero_infinity=True,
                        batch_first=True)
    loss.sum().backward()
    torch.cuda.synchronize()
    assert torch.all(guard == 7.0)
    cl_il = bad_il.clamp(max=T)
    cl_tl = bad_tl.clamp(max=S)
    cl_tg = bad_tg.clamp(0, V - 1)
    want, _ = oc.ctc_loss(x.double().numpy(), cl_tg.numpy(), cl_il.numpy(), cl_tl.numpy(), 0, "none", True)
    np.testing.assert_allclose(loss.detach().cpu().double().numpy(), want, rtol=1e-5, atol=1e-6)
    assert torch.isfinite(xd.grad).all()


def test_ctc_mean_and_nonfinite_counter():
    """cfm_ctc_mean: torch.nn.CTCLoss's reduction='mean' (mean_b nll_b / max(L_b, 1)) in one launch, and its
    optional device counter of non-finite results (the bench's bad-step count)."""
    from nn_conformer_for_speech_recognition_amd import ops
    cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
    nll = torch.tensor([3.0, 5.5, 0.25, 7.0], device=DEV)
    tl = torch.tensor([2, 0, 1, 4], dtype=torch.int32, device=DEV)
    out = ops.ctc_mean(nll, tl, cnt)
    ref = (nll.double().cpu() / tl.clamp(min=1).double().cpu()).mean().item()
    assert abs(out.item() - ref) <= 1e-6 * abs(ref)
    assert cnt.item() == 0
    for bad in (float("nan"), float("inf")):
        nb = nll.clone()
        nb[2] = bad
        out = ops.ctc_mean(nb, tl, cnt)
        assert not torch.isfinite(out).item()
    assert cnt.item() == 2
    big = torch.rand(700, device=DEV) * 50          # more utterances than the kernel's 256 threads
    tb = torch.randint(0, 40, (700,), dtype=torch.int32, device=DEV)
    ref = (big.double().cpu() / tb.clamp(min=1).double().cpu()).mean().item()
    assert abs(ops.ctc_mean(big, tb).item() - ref) <= 1e-5 * abs(ref)


def test_ctc_long_targets_vs_torch():
    """The wave-pipelined recursion at its limits: S = 2 Smax + 1 up to 1021 states (16 waves, the LDS edge rings
    wrapping over hundreds of frames), mixed target lengths so utterances run different wave counts (1 .. 16), both
    directions (loss and logits gradient) against torch fp64 -- as test_ctc_bench_shape_vs_torch, held to 2x the
    distance of torch's own fp32 CTC from fp64."""
    g = torch.Generator().manual_seed(21)
    B, T, V, U = 6, 1200, 64, 510
    x = torch.randn(B, T, V, generator=g)
    tgt = torch.randint(1, V, (B, U), generator=g)
    tgt[1, 10:20] = 5                    # repeats: states that cannot skip
    il = torch.tensor([T, T, 1100, 700, 300, T])
    tl = torch.tensor([U, 500, 260, 31, 100, 1])
    xr = x.double().clone().requires_grad_()
    ref = F.ctc_loss(F.log_softmax(xr, -1).transpose(0, 1), tgt, il, tl, reduction="sum", zero_infinity=True)
    ref.backward()
    x32 = x.clone().requires_grad_()
    F.ctc_loss(F.log_softmax(x32, -1).transpose(0, 1), tgt, il, tl, reduction="sum", zero_infinity=True).backward()
    xd = x.to(DEV).requires_grad_()
    loss = ctc.ctc_loss(xd, tgt.to(DEV), il.to(DEV), tl.to(DEV), reduction="none", zero_infinity=True,
                        batch_first=True)
    loss.sum().backward()
    ref_none = F.ctc_loss(F.log_softmax(x.double(), -1).transpose(0, 1), tgt, il, tl, reduction="none",
                          zero_infinity=True)
    np.testing.assert_allclose(loss.detach().cpu().double().numpy(), ref_none.numpy(), rtol=2e-5)
    err_ref32 = (x32.grad.double() - xr.grad).abs().max().item()
    err = (xd.grad.cpu().double() - xr.grad).abs().max().item()
    assert err <= 2 * err_ref32 + 1e-6, (err, err_ref32)


@pytest.mark.parametrize("mask", [1, 2, 3])
def test_ctc_recursion_abort_is_visible(mask):
    """A recursion that gives up a wait (forced here per direction) must not leave a finite loss with a wrong
    gradient: the aborted utterances' nll and logits gradient are NaN, the others untouched, and the abort counter
    counts them (the beta workgroup's abort used to reach nothing)."""
    from nn_conformer_for_speech_recognition_amd import _lib
    x, tgt, il, tl = _case(3)
    cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
    _lib.call("cfm_ctc_bind_abort_counter", _lib.ptr(cnt))
    _lib.call("cfm_ctc_set_debug", mask)
    try:
        xd = x.to(DEV).requires_grad_()
        loss = ctc.ctc_loss(xd, tgt.to(DEV), il.to(DEV), tl.to(DEV), reduction="none", zero_infinity=True,
                            batch_first=True)
        loss.sum().backward()
        torch.cuda.synchronize()
    finally:
        _lib.call("cfm_ctc_set_debug", 0)
        _lib.call("cfm_ctc_bind_abort_counter", None)
    B = x.shape[0]
    assert torch.isnan(loss).all().item(), loss           # every utterance forced (Tb > 0 for all)
    assert torch.isnan(xd.grad[0]).any().item()
    assert int(cnt.item()) == B
    # the debug mask off again: finite
    xd2 = x.to(DEV).requires_grad_()
    l2 = ctc.ctc_loss(xd2, tgt.to(DEV), il.to(DEV), tl.to(DEV), reduction="none", zero_infinity=True,
                      batch_first=True)
    assert torch.isfinite(l2).all().item()
