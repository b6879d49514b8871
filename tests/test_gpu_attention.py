"""MFMA attention kernels (cfm_attn_fwd / cfm_attn_bwd, bf16) against a torch fp32 reference of
nn.MultiheadAttention's core: softmax(q k^T / sqrt(dk) + key_padding_mask) v, ragged lengths.
Both kernel families are checked: whole-head with the wave-per-key-block dK/dV (default) and tiled (mode 1);
the two must agree with each other under dropout (same counter-based masks; the dQ, dK and dV slices compared
separately), and the masks themselves are read back exactly and checked against a numpy restatement of the hash."""
import numpy as np
import pytest
import torch

from nn_conformer_for_speech_recognition_amd import _lib, ops
from tests import dropout_hash as dh

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture
def attn_mode():
    yield lambda m: _lib.call("cfm_attn_set_mode", m)
    _lib.call("cfm_attn_set_mode", 0)


def _ref(qkv, lens, B, T, H, dk, do):
    x = qkv.float().view(B, T, 3, H, dk).requires_grad_()
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / dk ** 0.5
    mask = torch.arange(T, device=qkv.device)[None, :] >= lens[:, None].long()
    s = s.masked_fill(mask[:, None, None, :], float("-inf"))
    o = (s.softmax(-1) @ v).transpose(1, 2).reshape(B * T, H * dk)
    o.backward(do.float())
    return o.detach(), x.grad.view(B * T, 3 * H * dk)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("B,T,H", [(3, 373, 2), (2, 64, 4), (2, 97, 1)])
def test_attention_vs_torch(attn_mode, mode, B, T, H):
    attn_mode(mode)
    dk = 64
    g = torch.Generator().manual_seed(T + 7 * H + mode)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to(DEV, torch.bfloat16)
    lens = torch.tensor([T] + [max(1, T - 13 * (i + 1)) for i in range(B - 1)], dtype=torch.int32, device=DEV)
    do = torch.randn(B * T, H * dk, generator=g).to(DEV, torch.bfloat16)
    o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk)
    dqkv, _, _, _ = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk)
    ro, rg = _ref(qkv, lens, B, T, H, dk, do)
    assert _rel(o.float(), ro) < 1e-2
    assert _rel(dqkv.float(), rg) < 2e-2


@pytest.mark.parametrize("B,T,H,dk,lens", [(2, 373, 4, 64, [373, 250]), (3, 97, 2, 64, [97, 40, 1]),
                                         (2, 373, 4, 36, [373, 301]), (1, 384, 2, 64, [384]), (2, 130, 2, 64, [130, 65])])
@pytest.mark.parametrize("drop_p", [0.0, 0.1])
def test_dq_from_stored_ds_matches_recompute(attn_mode, B, T, H, dk, lens, drop_p):
    """Whole-head backward: dQ from the dS^T the dK/dV kernel stores (default with the full workspace) against the
    recomputing dQ kernel (cfm_attn_set_mode bit 10): dK / dV bit-identical (the same kernel, plus stores), dQ equal
    up to the bf16 rounding of the stored dS (the recomputing kernel rounds the same values, in another order);
    ragged lengths incl. a length-1 utterance and keys past len; dk 36 (Conformer-S); T 384 (Tq = T) and 130."""
    g = torch.Generator().manual_seed(T + dk + H)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to(DEV, torch.bfloat16)
    lt = torch.tensor(lens, dtype=torch.int32, device=DEV)
    do = torch.randn(B * T, H * dk, generator=g).to(DEV, torch.bfloat16)
    o, lse = ops.attn_fwd(qkv, lt, B, T, H, dk, drop_p=drop_p, seed=3)
    outs = []
    for m in (1024, 0):
        attn_mode(m)
        dqkv, _, _, _ = ops.attn_bwd(qkv, o, do, lse, lt, B, T, H, dk, drop_p=drop_p, seed=3)
        outs.append(dqkv.float().view(B * T, 3, H * dk))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][:, 1:], outs[1][:, 1:])
    assert _rel(outs[1][:, 0], outs[0][:, 0]) < 5e-3
    assert torch.isfinite(outs[1]).all()


def test_attention_kernels_agree_under_dropout(attn_mode):
    B, T, H, dk = 2, 373, 2, 64
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to(DEV, torch.bfloat16)
    lens = torch.tensor([T, 300], dtype=torch.int32, device=DEV)
    do = torch.randn(B * T, H * dk, generator=g).to(DEV, torch.bfloat16)
    outs = []
    for mode in (0, 1):
        attn_mode(mode)
        o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=9)
        dqkv, _, _, _ = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=0.1, seed=9)
        outs.append((o.float(), dqkv.float()))
    HD = H * dk
    for o, d in outs[1:]:
        assert _rel(o, outs[0][0]) < 1e-2
        for sl in range(3):      # dQ, dK, dV: a mask that differs on ~10 % of the entries fails these
            assert _rel(d[:, sl * HD:(sl + 1) * HD], outs[0][1][:, sl * HD:(sl + 1) * HD]) < 1e-2


def test_rowdot_epilogue_feeds_attention_bwd():
    """D = rowsum(dO * O) per head from the out-projection dgrad GEMM's epilogue (cfm_gemm_desc.rowdot_*)
    equals the separate D pass, and cfm_attn_bwd_with_d reproduces cfm_attn_bwd."""
    B, T, H, dk = 3, 97, 8, 64
    g = torch.Generator().manual_seed(21)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to(DEV, torch.bfloat16)
    lens = torch.tensor([T, 80, 50], dtype=torch.int32, device=DEV)
    o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=4)
    g4 = torch.randn(B * T, H * dk, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(H * dk, H * dk, generator=g) * 0.05).to(DEV, torch.bfloat16)
    D = torch.empty(B * H * T, device=DEV)
    do = ops.linear_dgrad(g4, w, wt=w.t().contiguous(), rowdot=(o, D, T))
    ref = (do.float() * o.float()).view(B, T, H, dk).sum(-1).permute(0, 2, 1).reshape(-1)
    torch.cuda.synchronize()
    assert _rel(D, ref) < 1e-5
    d1, _, _, _ = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=0.1, seed=4)
    d2, _, _, _ = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=0.1, seed=4, D=D)
    assert _rel(d2.float(), d1.float()) < 1e-3


# ------------------------------------------------------------------------------------ relative positions
def _ref_rel(qkv, pos, pu, pv, lens, B, T, H, dk, do):
    """fp32 torch restatement of transformers' rel-pos attention core (modeling_wav2vec2_conformer.py:528-565):
    scores = ((q+u) k^T + rel_shift((q+v) p^T)) / sqrt(dk), bd[i, j] uses p row (T-1) - i + j."""
    x = qkv.float().view(B, T, 3, H, dk).requires_grad_()
    P = pos.float().view(2 * T - 1, H, dk).requires_grad_()
    u = pu.float().view(H, dk).requires_grad_()
    v = pv.float().view(H, dk).requires_grad_()
    q, k, vv = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    ac = (q + u[None, :, None, :]) @ k.transpose(-1, -2)
    full = (q + v[None, :, None, :]) @ P.permute(1, 2, 0)[None]          # (B, H, T, 2T-1)
    ar = torch.arange(T, device=qkv.device)
    idx = (T - 1 - ar[:, None] + ar[None, :]).expand(B, H, T, T)
    s = (ac + full.gather(-1, idx)) / dk ** 0.5
    mask = ar[None, :] >= lens[:, None].long()
    s = s.masked_fill(mask[:, None, None, :], float("-inf"))
    o = (s.softmax(-1) @ vv).transpose(1, 2).reshape(B * T, H * dk)
    o.backward(do.float())
    return o.detach(), x.grad.view(B * T, 3 * H * dk), P.grad.view(2 * T - 1, H * dk), u.grad.reshape(-1), \
        v.grad.reshape(-1)


def _rel_case(B, T, H, dk, lens, seed):
    g = torch.Generator().manual_seed(seed)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to(DEV, torch.bfloat16)
    pos = (0.5 * torch.randn(2 * T - 1, H * dk, generator=g)).to(DEV, torch.bfloat16)
    pu = (0.3 * torch.randn(H * dk, generator=g)).to(DEV)
    pv = (0.3 * torch.randn(H * dk, generator=g)).to(DEV)
    do = torch.randn(B * T, H * dk, generator=g).to(DEV, torch.bfloat16)
    ln = torch.tensor(lens, dtype=torch.int32, device=DEV)
    return qkv, pos, pu, pv, do, ln


@pytest.mark.parametrize("B,T,H,dk,lens", [
    (3, 373, 2, 64, [373, 300, 41]),       # the metric's T_enc, ragged
    (1, 1498, 2, 64, [1498]),              # config 5: 60 s long-form (T_enc = 1498)
    (2, 1498, 1, 64, [1498, 1001]),
    (2, 97, 4, 36, [97, 60]),              # Conformer-S head dim (zero-padded to 64)
    (2, 64, 1, 64, [64, 1]),
])
def test_rel_attention_vs_torch(B, T, H, dk, lens):
    """MFMA rel-pos kernels (attention_rel.hip) vs the fp32 torch restatement: outputs and every
    gradient (q/k/v, projected table p, pos_bias_u, pos_bias_v).  Tolerance: relative L2 1e-2 (o),
    2e-2 (dqkv, dpos), 3e-2 (du, dv: sums over all queries of bf16-rounded dS products)."""
    qkv, pos, pu, pv, do, ln = _rel_case(B, T, H, dk, lens, T + H)
    o, lse = ops.attn_fwd(qkv, ln, B, T, H, dk, pos, pu, pv)
    dqkv, dpos, dpu, dpv = ops.attn_bwd(qkv, o, do, lse, ln, B, T, H, dk, pos, pu, pv)
    ro, rg, rp, ru, rv = _ref_rel(qkv, pos, pu, pv, ln, B, T, H, dk, do)
    torch.cuda.synchronize()
    assert _rel(o.float(), ro) < 1e-2
    assert _rel(dqkv.float(), rg) < 2e-2
    assert _rel(dpos, rp) < 2e-2
    assert _rel(dpu, ru) < 3e-2
    assert _rel(dpv, rv) < 3e-2
    # per valid query row, worst max-abs error relative to the row's max (a bad row cannot hide in the L2)
    ob = o.float().view(B, T, -1).cpu()
    rb = ro.view(B, T, -1).cpu()
    for b, n in enumerate(lens):
        d = (ob[b, :n] - rb[b, :n]).abs().amax(-1) / rb[b, :n].abs().amax(-1).clamp_min(1e-30)
        assert d.max().item() < 5e-2, (b, d.argmax().item())


def test_rel_attention_mfma_matches_simt_under_dropout(attn_mode):
    """Same counter-based attention-dropout masks on both rel-pos paths: MFMA (default) and the SIMT kernels
    (cfm_attn_set_mode bit 4), fwd + every gradient."""
    B, T, H, dk = 2, 150, 2, 64
    qkv, pos, pu, pv, do, ln = _rel_case(B, T, H, dk, [150, 111], 3)
    outs = []
    for mode in (0, 16):
        attn_mode(mode)
        o, lse = ops.attn_fwd(qkv, ln, B, T, H, dk, pos, pu, pv, drop_p=0.15, seed=77)
        g = ops.attn_bwd(qkv, o, do, lse, ln, B, T, H, dk, pos, pu, pv, drop_p=0.15, seed=77)
        outs.append((o.float(), g[0].float(), g[1], g[2], g[3]))
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert _rel(a, b) < 3e-2


@pytest.mark.parametrize("B,T,H,lens", [(2, 1498, 3, [1498, 1001]), (3, 373, 2, [373, 300, 41]), (2, 64, 1, [64, 1]),
                                        (9, 130, 2, [130] * 8 + [77])])
def test_rel_dpos_xcd_kernel_matches_round4(attn_mode, B, T, H, lens):
    """The round-5 dpos kernel (128 relative rows per workgroup, (b, h) pairs dealt to XCDs, dword-funnel band
    loads, masks on edge tiles only) == the round-4 kernel (cfm_attn_set_mode bit 7) bit for bit: the same MFMA
    k-steps over the same i order, the extra leading rows contribute exact zeros.  B*H = 18 pads the XCD deal."""
    dk = 64
    qkv, pos, pu, pv, do, ln = _rel_case(B, T, H, dk, lens, 5)
    outs = []
    for mode in (0, 128):
        attn_mode(mode)
        o, lse = ops.attn_fwd(qkv, ln, B, T, H, dk, pos, pu, pv, drop_p=0.1, seed=11)
        outs.append(ops.attn_bwd(qkv, o, do, lse, ln, B, T, H, dk, pos, pu, pv, drop_p=0.1, seed=11)[1])
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B,T,H,lens", [(2, 373, 2, [373, 250]), (2, 1498, 2, [1498, 1001]), (3, 130, 2, [130, 77, 1])])
@pytest.mark.parametrize("drop_p", [0.0, 0.1])
def test_rel_dq_from_stored_ds_matches_recompute(attn_mode, B, T, H, lens, drop_p):
    """Rel-pos backward: dQ from the dS the dK/dV kernel stores (attn_rel_bwd_dqs_kernel, default; its band scatter is
    explicit 2-byte LDS stores) against the recomputing dQ2 kernel (cfm_attn_set_mode bit 9): dK / dV and dpos
    bit-identical (the same kernels), dQ and the u / v gradients equal up to the bf16 rounding of the stored dS;
    ragged lengths incl. a length-1 utterance, T 1498 (L60)."""
    dk = 64
    qkv, pos, pu, pv, do, ln = _rel_case(B, T, H, dk, lens, 13)
    o, lse = ops.attn_fwd(qkv, ln, B, T, H, dk, pos, pu, pv, drop_p=drop_p, seed=5)
    outs = []
    for m in (512, 0):
        attn_mode(m)
        dqkv, dpos, dpu, dpv = ops.attn_bwd(qkv, o, do, lse, ln, B, T, H, dk, pos, pu, pv, drop_p=drop_p, seed=5)
        outs.append((dqkv.float().view(B * T, 3, H * dk), dpos.float(), dpu.float(), dpv.float()))
    torch.cuda.synchronize()
    (r, rpos, ru, rv), (n, npos, nu, nv) = outs
    assert torch.isfinite(n).all() and torch.isfinite(npos).all()
    assert torch.equal(r[:, 1:], n[:, 1:])
    assert torch.equal(rpos, npos)
    assert _rel(n[:, 0], r[:, 0]) < 5e-3
    assert _rel(nu, ru) < 5e-3 and _rel(nv, rv) < 5e-3


# ------------------------------------------------------------------------------------ dropout masks, read back
def _keep(B, T, H, p, seed):
    """numpy restatement of the attention-dropout keep mask (cfm_common.h attn_mix / drop_key, attn_common.h
    didx): element (b, h, i, j) keeps iff the 16-bit half (j & 1) of attn_mix(((bh T + i) T2 + j/2) + key) >= thr,
    T2 = (T rounded up to even) / 2, key = lowbias32-derived drop_key(seed, 0).  Returns (B, H, T, T) bool."""
    key = dh.drop_key(seed)
    thr = dh.drop_thr(p)
    T2 = (T + (T & 1)) >> 1
    bh = np.arange(B * H, dtype=np.uint64)[:, None, None]
    i = np.arange(T, dtype=np.uint64)[None, :, None]
    j = np.arange(T, dtype=np.uint64)[None, None, :]
    hs = dh.attn_mix((((bh * T + i) * T2 + j // 2) + key) & 0xFFFFFFFF)
    half = np.where(j % 2 == 0, hs & 0xFFFF, hs >> 16)
    return (half >= thr).reshape(B, H, T, T)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("T,seed", [(64, 9), (63, (1 << 40) + 5), (37, 77)])
def test_dropout_masks_read_back(attn_mode, mode, T, seed):
    """q = k = 0 makes P uniform (1 / T); V = identity rows makes o[i, j] = keep(i, j) / ((1 - p) T), and dO =
    identity rows makes dV[j, i] = the same (P^T dO): both masks -- the forward's query-major one and the dK/dV
    kernel's key-major one -- come back exactly and must equal the numpy restatement of the hash."""
    attn_mode(mode)
    B, H, dk, p = 2, 2, 64, 0.1
    qkv = torch.zeros(B, T, 3, H, dk)
    eye = torch.eye(T, dk)
    qkv[:, :, 2] = eye[None, :, None, :]
    qkv = qkv.reshape(B * T, 3 * H * dk).to(DEV, torch.bfloat16)
    lens = torch.full((B,), T, dtype=torch.int32, device=DEV)
    o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=p, seed=seed)
    do = eye[None, :, None, :].expand(B, T, H, dk).reshape(B * T, H * dk).to(DEV, torch.bfloat16).contiguous()
    dqkv, _, _, _ = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=p, seed=seed)
    torch.cuda.synchronize()
    ref = _keep(B, T, H, p, seed)                                                   # (B, H, i, j)
    got_f = (o.float().view(B, T, H, dk)[..., :T] > 0).permute(0, 2, 1, 3).cpu().numpy()
    np.testing.assert_array_equal(got_f, ref)
    dv = dqkv.float().view(B, T, 3, H, dk)[:, :, 2, :, :T]                          # (B, j, H, i)
    got_b = (dv > 0).permute(0, 2, 3, 1).cpu().numpy()
    np.testing.assert_array_equal(got_b, ref)
    val = o.float().view(B, T, H, dk)[..., :T][torch.from_numpy(ref).permute(0, 2, 1, 3).to(DEV)]
    assert torch.allclose(val, torch.full_like(val, 1.0 / ((1 - p) * T)), rtol=1e-2)
    assert 0.85 < ref.mean() < 0.95


def test_rel_dpos_bf16_output_is_the_cast():
    """cfm_attn_bwd_ex with dtype_dpos bf16: dpos written in the compute dtype by the column reduction equals the
    fp32 dpos cast to bf16 (the same fp32 sums, rounded as cfm_cast), at the L60 width and at a width below the
    few-rows kernel's range (the reduce-in-place + cast fallback); every other output unchanged."""
    for (B, T, H, lens) in [(2, 1498, 2, [1498, 1001]), (2, 97, 4, [97, 60])]:
        qkv, pos, pu, pv, do, ln = _rel_case(B, T, H, 64, lens, 13)
        o, lse = ops.attn_fwd(qkv, ln, B, T, H, 64, pos, pu, pv, drop_p=0.1, seed=3)
        ref = ops.attn_bwd(qkv, o, do, lse, ln, B, T, H, 64, pos, pu, pv, drop_p=0.1, seed=3)
        got = ops.attn_bwd(qkv, o, do, lse, ln, B, T, H, 64, pos, pu, pv, drop_p=0.1, seed=3, dpos_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        assert got[1].dtype == torch.bfloat16
        assert torch.equal(got[1], ops.cast(ref[1], torch.bfloat16))
        for a, b in zip((got[0], got[2], got[3]), (ref[0], ref[2], ref[3])):
            assert torch.equal(a, b)
