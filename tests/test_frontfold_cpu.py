"""CPU checks of the folded 'frame'-mode front-end (frontfold.hip): the algebra the kernels implement, restated
in fp64 torch (the two convolutions of lib/convsubsampling.py:41-43 followed by the per-frame Linear equal ONE
Ke x Ke / stride-Se window map, forward and all six parameter gradients), and the host-side geometry
(cfm_ffold_geometry: no GPU work) against the reference's out_size arithmetic (convsubsampling.py:24-32)."""
import pytest
import torch
import torch.nn.functional as F

from nn_conformer_for_speech_recognition_amd import ops


def compose(w1, b1, w2, b2, wp, bp, s1, s2, F2, C2):
    """W_eff (C2, Ke, Ke), b_eff, Wfull (D, Ke[time], Fr[mel]), bfull -- the formulas of frontfold.hip."""
    C1, k1, k2 = w1.shape[0], w1.shape[-1], w2.shape[-1]
    Ke, Se = k1 + (k2 - 1) * s1, s1 * s2
    weff = torch.zeros(C2, Ke, Ke, dtype=torch.float64)
    for a in range(k2):
        for b in range(k2):
            weff[:, s1 * a:s1 * a + k1, s1 * b:s1 * b + k1] += torch.einsum("dc,chw->dhw", w2[:, :, a, b], w1[:, 0])
    beff = b2 + torch.einsum("dcab,c->d", w2, b1)
    D = wp.shape[0]
    Fr = Se * (F2 - 1) + Ke
    wfull = torch.zeros(D, Ke, Fr, dtype=torch.float64)
    wpr = wp.view(D, F2, C2)
    for f2 in range(F2):
        # Wfull[o][f][Se f2 + e] += sum_c2 Wp[o][f2, c2] W_eff[c2][e][f]
        wfull[:, :, Se * f2:Se * f2 + Ke] += torch.einsum("oc,cef->ofe", wpr[:, f2], weff)
    bfull = bp + torch.einsum("ofc,c->o", wpr, beff)
    return weff, beff, wfull, bfull


@pytest.mark.parametrize("B,Fb,T,C1,C2,D", [(2, 80, 61, 16, 8, 12), (1, 40, 45, 8, 16, 5)])
def test_fold_identity_fp64(B, Fb, T, C1, C2, D):
    torch.manual_seed(0)
    w1 = torch.randn(C1, 1, 7, 7, dtype=torch.float64)
    b1 = torch.randn(C1, dtype=torch.float64)
    w2 = torch.randn(C2, C1, 3, 3, dtype=torch.float64)
    b2 = torch.randn(C2, dtype=torch.float64)
    x = torch.randn(B, Fb, T, dtype=torch.float64)
    h = F.conv2d(F.conv2d(x.unsqueeze(1), w1, b1, stride=2), w2, b2, stride=2)
    _, _, F2, T2 = h.shape
    wp = torch.randn(D, F2 * C2, dtype=torch.float64)
    bp = torch.randn(D, dtype=torch.float64)
    ref = F.linear(h.permute(0, 3, 2, 1).reshape(B * T2, F2 * C2), wp, bp)
    weff, beff, wfull, bfull = compose(w1, b1, w2, b2, wp, bp, 2, 2, F2, C2)
    Ke, Se, Fr = 11, 4, wfull.shape[-1]
    # window view: rows (b, t2), columns (f, r) = x[b, r, Se t2 + f]
    win = torch.stack([x[:, :Fr, Se * t:Se * t + Ke].transpose(1, 2) for t in range(T2)], 1)   # (B, T2, Ke, Fr)
    y = win.reshape(B * T2, Ke * Fr) @ wfull.reshape(D, -1).T + bfull
    assert torch.allclose(y, ref, rtol=1e-10, atol=1e-9)
    # backward: G -> H = G^T X, S = colsum G; the contractions of frontfold.hip vs autograd
    G = torch.randn(B * T2, D, dtype=torch.float64)
    ps = [t.clone().requires_grad_() for t in (w1, b1, w2, b2, wp, bp)]
    hh = F.conv2d(F.conv2d(x.unsqueeze(1), ps[0], ps[1], stride=2), ps[2], ps[3], stride=2)
    F.linear(hh.permute(0, 3, 2, 1).reshape(B * T2, F2 * C2), ps[4], ps[5]).backward(G)
    Hm = (G.T @ win.reshape(B * T2, Ke * Fr)).view(D, Ke, Fr)       # H[o][f][r]
    S = G.sum(0)
    wpr = wp.view(D, F2, C2)
    dweff = torch.zeros(C2, Ke, Ke, dtype=torch.float64)
    dwp = torch.zeros(D, F2, C2, dtype=torch.float64)
    for f2 in range(F2):
        hsl = Hm[:, :, Se * f2:Se * f2 + Ke]                          # (o, f, e)
        dweff += torch.einsum("oc,ofe->cef", wpr[:, f2], hsl)
        dwp[:, f2] = torch.einsum("cef,ofe->oc", weff, hsl) + S[:, None] * beff[None]
    dbeff = torch.einsum("ofc,o->c", wpr, S)
    dw2 = torch.zeros_like(w2)
    dw1 = torch.zeros_like(w1)
    for a in range(3):
        for b in range(3):
            blk = dweff[:, 2 * a:2 * a + 7, 2 * b:2 * b + 7]           # (c2, kh, kw)
            dw2[:, :, a, b] = torch.einsum("chw,dhw->dc", w1[:, 0], blk) + dbeff[:, None] * b1[None]
            dw1[:, 0] += torch.einsum("dc,dhw->chw", w2[:, :, a, b], blk)
    db1 = torch.einsum("dcab,d->c", w2, dbeff)
    for got, p in zip((dw1, db1, dw2, dbeff, dwp.reshape(D, -1), S), ps):
        assert torch.allclose(got, p.grad, rtol=1e-9, atol=1e-8)


def test_geometry_host_call():
    """cfm_ffold_geometry at BASELINE configs[1] (80 x 1501 mels, 512 / 128 channels, D 512), bf16 hi + lo."""
    g = ops.ffold_geometry(32, 80, 1501, 512, 128, 512, 7, 2, 3, 2, torch.bfloat16, True)
    assert (g.F2, g.T2, g.Ke, g.Se) == (18, 373, 11, 4)
    assert (g.Fp, g.Cx, g.Kp, g.lda) == (80, 160, 1792, 640)
    assert g.Kp % 64 == 0 and g.Kp >= g.Ke * g.Cx
    # every view row of the forward stays inside its utterance slot; the padded rows of the backward view
    # stay inside the allocation
    assert (g.T2 - 1) * g.lda + g.Kp <= g.Tslot * g.Cx
    assert g.Tslot == g.Se * g.T2p and (g.B * g.T2p - 1) * g.lda + g.Kp <= g.xt_elems
    assert g.Se * (g.T2 - 1) + g.Ke <= 1501
    g32 = ops.ffold_geometry(2, 80, 161, 512, 128, 144, 7, 2, 3, 2, torch.float32)
    assert (g32.Cx, g32.Kp, g32.lda) == (80, 880, 320)
    # the reference's out_size arithmetic (convsubsampling.py:24-32)
    h, w = 80, 161
    for k, s in ((7, 2), (3, 2)):
        h, w = (h - k + s) // s, (w - k + s) // s
    assert (g32.F2, g32.T2) == (h, w)
