"""MFMA attention kernels (cfm_attn_fwd / cfm_attn_bwd, bf16) against a torch fp32 reference of
nn.MultiheadAttention's core: softmax(q k^T / sqrt(dk) + key_padding_mask) v, ragged lengths.
Every kernel family is checked: whole-head (default), tiled (mode 1), wave-per-key-block dK/dV
(mode 8); and the three must agree with each other under dropout (same counter-based masks)."""
import pytest
import torch

from nn_conformer_for_speech_recognition_amd import _lib, ops

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


@pytest.mark.parametrize("mode", [0, 1, 8])
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


def test_attention_kernels_agree_under_dropout(attn_mode):
    B, T, H, dk = 2, 373, 2, 64
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(B * T, 3 * H * dk, generator=g).to(DEV, torch.bfloat16)
    lens = torch.tensor([T, 300], dtype=torch.int32, device=DEV)
    do = torch.randn(B * T, H * dk, generator=g).to(DEV, torch.bfloat16)
    outs = []
    for mode in (0, 1, 8):
        attn_mode(mode)
        o, lse = ops.attn_fwd(qkv, lens, B, T, H, dk, drop_p=0.1, seed=9)
        dqkv, _, _, _ = ops.attn_bwd(qkv, o, do, lse, lens, B, T, H, dk, drop_p=0.1, seed=9)
        outs.append((o.float(), dqkv.float()))
    for o, d in outs[1:]:
        assert _rel(o, outs[0][0]) < 1e-2
        assert _rel(d, outs[0][1]) < 2e-2


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
