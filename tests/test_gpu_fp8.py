"""fp8 (e4m3fn, OCP) path of BASELINE.json configs[4] -- no reference counterpart (the reference is fp32):
per-tensor quantisation (cfm_quant_fp8, power-of-two scales) and the block-scaled-MFMA GEMM (v_mfma_scale_f32_32x32x64_f8f6f4,
unit block scales, per-tensor dequantisation in the epilogue).

Tolerances: the GEMM against an fp64 product of the SAME quantised operands -- relative L2 5e-5 with fp32
output (exact fp8 products, fp32 accumulation) and 8e-3 with bf16 output; the quantisation itself
bit-exact against torch's float8_e4m3fn conversion of x * 2^k (the largest k with amax * 2^k <= 448); the whole fp8 path against the fp32
product of the unquantised operands: relative L2 <= 6e-2 (e4m3's 3 mantissa bits)."""
import pytest
import torch

from nn_conformer_for_speech_recognition_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_quant_fp8_bit_exact(dt):
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(1000, 264, generator=g) * 3).to(dt)
    x[3, 7] = -17.25
    y, sc = ops.quant_fp8(x.to(DEV))
    amax = x.float().abs().max().item()
    k = 0                                           # largest k with amax * 2^k <= 448
    while amax * 2.0 ** (k + 1) <= 448.0:
        k += 1
    while amax * 2.0 ** k > 448.0:
        k -= 1
    assert sc.item() == 2.0 ** -k
    ref = (x.float() * 2.0 ** k).to(torch.float8_e4m3fn)
    assert torch.equal(y.cpu().view(torch.uint8), ref.view(torch.uint8))


@pytest.mark.parametrize("M,N,K", [(11936, 2048, 512), (11936, 512, 2048), (1000, 1536, 512), (77, 512, 128)])
def test_fp8_gemm_vs_fp64_of_quantised(M, N, K):
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (0.05 * torch.randn(N, K, generator=g)).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    xq, sx = ops.quant_fp8(x)
    wq, sw = ops.quant_fp8(w)
    ref = (xq.cpu().double() * sx.item()) @ (wq.cpu().double() * sw.item()).t() + b.cpu().double()
    y32 = ops.linear(xq, wq, b, out_dtype=torch.float32, x_scale=sx, w_scale=sw)
    assert _rel(y32, ref) < 5e-5
    y16 = ops.linear(xq, wq, b, x_scale=sx, w_scale=sw)
    assert y16.dtype == torch.bfloat16 and _rel(y16.float(), ref) < 8e-3
    full = x.double().cpu() @ w.double().cpu().t() + b.cpu().double()
    assert _rel(y32, full) < 6e-2


def test_fp8_gemm_silu_dropout_epilogue():
    """The FFN up-projection's epilogue (bias + SiLU + dropout + saved pre-activation) on fp8 operands equals
    the bf16 kernel's epilogue applied to the same (dequantised) product."""
    M, N, K = 2000, 1024, 256
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (0.05 * torch.randn(N, K, generator=g)).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    xq, sx = ops.quant_fp8(x)
    wq, sw = ops.quant_fp8(w)
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y = ops.linear(xq, wq, b, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=5, x_scale=sx, w_scale=sw)
    z = (xq.float() * sx) @ (wq.float() * sw).t() + b
    assert _rel(pre.float(), z) < 8e-3
    keep = (y.float() != 0)
    frac = keep.float().mean().item()
    assert 0.88 < frac < 0.92
    want = torch.nn.functional.silu(pre.float()) / 0.9
    assert _rel(y.float()[keep], want[keep]) < 1e-2


@pytest.mark.parametrize("T,lens", [(373, [373, 290]), (1498, [1498, 1201])])
def test_conformer_fp8_forward_vs_fp32_oracle(T, lens):
    """Conformer-L dims (d 512, 8 heads, ffn 2048), ragged lengths, rel-pos (configs[4]'s attention), with the
    forward FFN / QKV / out-projection GEMMs on fp8 and the backward in bf16, against the fp32 oracle -- at 15 s
    (T 373) and at configs[4]'s 60 s (T 1498).
    Tolerance (stated for the fp8 path): relative L2 5e-2 on the output, 1e-1 on input and weight gradients."""
    from nn_conformer_for_speech_recognition_amd.conformer import Conformer
    from oracle import conformer as oc
    torch.manual_seed(7)
    d, H, ffn, K, L, B = 512, 8, 2048, 31, 1, 2
    ref = oc.ConformerRef(d, H, ffn, L, K, 0.0, pos_enc="rel").train()
    with torch.no_grad():
        for n, prm in ref.named_parameters():
            if n.endswith("bias"):
                prm.normal_(0, 0.05)
    m = Conformer(d, H, ffn, L, K, 0.0, pos_enc="rel", compute_dtype=torch.bfloat16, fp8=True)
    m.load_state_dict(ref.state_dict())
    m = m.to(DEV).train()
    x = torch.randn(B, T, d)
    ln = torch.tensor(lens)
    xr = x.clone().requires_grad_()
    yr, _ = ref(xr, ln)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    xd = x.to(DEV).requires_grad_()
    y, _ = m(xd, ln.to(DEV))
    y.backward(gy.to(DEV))
    ey, ex = _rel(y.detach(), yr.detach()), _rel(xd.grad, xr.grad)
    print("fp8 conformer rel err: y", ey, "dx", ex)
    assert ey < 5e-2 and ex < 1e-1
    rp = dict(ref.named_parameters())
    for n, prm in m.named_parameters():
        if n.endswith("conv_module.sequential.2.bias"):
            continue
        assert _rel(prm.grad, rp[n].grad) < 1e-1 * (3 if "pos_bias" in n else 1), n


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_quant_fp8_batch_matches_per_tensor(dt):
    """cfm_quant_fp8_batch (ops.Quant8Batch: the per-step fp8 weight copies, two launches for the list) gives the
    same bytes and scales as cfm_quant_fp8 tensor by tensor (bit-exact; sizes with tails and one-block tensors)."""
    g = torch.Generator().manual_seed(11)
    shapes = [(2048, 512), (512, 2048), (1536, 512), (7, 13), (1, 8), (3000, 1)]
    srcs = [(torch.randn(*s, generator=g) * (10.0 ** (i - 2))).to(DEV, dt).contiguous() for i, s in enumerate(shapes)]
    qb = ops.Quant8Batch(srcs)
    for _ in range(2):                       # refresh twice: persistent outputs overwritten in place
        outs = qb.refresh()
    for x, (y, sc) in zip(srcs, outs):
        y_ref, sc_ref = ops.quant_fp8(x)
        assert torch.equal(sc, sc_ref), (x.shape, sc.item(), sc_ref.item())
        assert torch.equal(y.view(torch.uint8), y_ref.view(torch.uint8)), x.shape


# ------------------------------------------------------------------------------------------- MX block scaling
def _mx_ref(x):
    """numpy/torch restatement of cfm_quant_mx: per 32-element block of a row, k = the largest integer with
    amax * 2^k <= 448 (0 for an all-zero block, clamped to [-126, 126]), y = e4m3(x * 2^k), s = 127 - k."""
    xf = x.float().cpu()
    rows, K = xf.shape
    blk = xf.view(rows, K // 32, 32)
    amax = blk.abs().amax(-1).double()
    m, e = torch.frexp(amax)                       # amax = m * 2^e, m in [0.5, 1)
    k = torch.where(2 * m <= 1.75, 8 - (e - 1), 7 - (e - 1)).clamp(-126, 126)
    k = torch.where(amax > 0, k, torch.zeros_like(k))
    y = (blk.double() * torch.pow(2.0, k.double())[..., None]).float().view(rows, K).to(torch.float8_e4m3fn)
    return y, (127 - k).to(torch.uint8)


def _mx_deq(y, s):
    yf = y.cpu().float().view(y.shape[0], -1, 32).double()
    return (yf * torch.pow(2.0, s.cpu().double() - 127)[..., None]).view(y.shape[0], -1)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_quant_mx_bit_exact(dt):
    """cfm_quant_mx (one pass, e8m0 scale per 32 elements) bit-exact against torch's float8_e4m3fn conversion of
    x * 2^k per block; rows with very different magnitudes, an all-zero block, and the dequantised view."""
    g = torch.Generator().manual_seed(2)
    x = (torch.randn(1000, 512, generator=g) * torch.logspace(-6, 6, 1000)[:, None]).to(dt)
    x[5, 32:64] = 0
    x[7, 3] = -17.25
    y, s = ops.quant_mx(x.to(DEV))
    yr, sr = _mx_ref(x)
    assert torch.equal(s.cpu(), sr)
    assert torch.equal(y.cpu().view(torch.uint8), yr.view(torch.uint8))
    deq = ops.dequant_mx(y, s)
    assert torch.equal(deq.cpu().double(), _mx_deq(y, s))
    assert _rel(deq, x.float()) < 6e-2


def test_quant_mx_batch_matches_per_tensor():
    g = torch.Generator().manual_seed(12)
    shapes = [(2048, 512), (512, 2048), (1536, 512), (7, 64), (1, 32)]
    srcs = [(torch.randn(*s, generator=g) * (10.0 ** (i - 2))).to(DEV).contiguous() for i, s in enumerate(shapes)]
    qb = ops.QuantMXBatch(srcs)
    for _ in range(2):
        outs = qb.refresh()
    for x, (y, s) in zip(srcs, outs):
        yr, sr = ops.quant_mx(x)
        assert torch.equal(s, sr) and torch.equal(y.view(torch.uint8), yr.view(torch.uint8)), x.shape


@pytest.mark.parametrize("M,N,K", [(11936, 2048, 512), (11936, 512, 2048), (1000, 1536, 512), (77, 512, 128),
                                   (300, 2048, 1024), (11984, 512, 512)])
def test_mx_gemm_vs_fp64_of_dequantised(M, N, K):
    """The MX GEMM (block scales inside v_mfma_scale_f32_32x32x64_f8f6f4) against an fp64 product of the SAME
    dequantised operands (rows of very different magnitudes, so the per-block scales matter): relative L2 5e-5 with
    fp32 output, 8e-3 with bf16; against the unquantised fp32 product 6e-2."""
    g = torch.Generator().manual_seed(M + 3 * N + K)
    x = (torch.randn(M, K, generator=g) * torch.logspace(-2, 2, K)[None, :]).to(DEV, torch.bfloat16)
    w = (0.05 * torch.randn(N, K, generator=g)).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    xq, sx = ops.quant_mx(x)
    wq, sw = ops.quant_mx(w)
    ref = _mx_deq(xq, sx) @ _mx_deq(wq, sw).t() + b.cpu().double()
    y32 = ops.linear(xq, wq, b, out_dtype=torch.float32, x_mx=sx, w_mx=sw)
    assert _rel(y32, ref) < 5e-5
    y16 = ops.linear(xq, wq, b, x_mx=sx, w_mx=sw)
    assert y16.dtype == torch.bfloat16 and _rel(y16.float(), ref) < 8e-3
    full = x.double().cpu() @ w.double().cpu().t() + b.cpu().double()
    assert _rel(y32, full) < 6e-2


def test_mx_gemm_epilogues():
    """The encoder's fp8 epilogues on MX operands (fast epilogue kinds): FFN up (bias + SiLU + dropout + saved
    pre-activation, bf16) and FFN down / out-projection (bias + dropout + 0.5 scale + fp32 residual) against the
    bf16-operand GEMM of the same dequantised values (identical dropout masks)."""
    g = torch.Generator().manual_seed(4)
    M = 3000
    for N, K, kind in ((2048, 512, "up"), (512, 2048, "down")):
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        w = (0.05 * torch.randn(N, K, generator=g)).to(DEV)
        b = torch.randn(N, generator=g).to(DEV)
        xq, sx = ops.quant_mx(x)
        wq, sw = ops.quant_mx(w)
        xd = ops.dequant_mx(xq, sx)
        wd = ops.dequant_mx(wq, sw)
        if kind == "up":
            pre8 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            y8 = ops.linear(xq, wq, b, act=ops.ACT_SILU, pre=pre8, drop_p=0.1, seed=5, x_mx=sx, w_mx=sw)
            pre32 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            y32 = ops.linear(xd, wd, b, act=ops.ACT_SILU, pre=pre32, drop_p=0.1, seed=5, out_dtype=torch.bfloat16)
            assert _rel(pre8.float(), pre32.float()) < 8e-3
            assert torch.equal(y8 == 0, y32 == 0)
            assert _rel(y8.float(), y32.float()) < 1e-2
        else:
            res = torch.randn(M, N, generator=g).to(DEV)
            y8 = ops.linear(xq, wq, b, out_dtype=torch.float32, drop_p=0.1, seed=6, out_scale=0.5, residual=res,
                            x_mx=sx, w_mx=sw)
            y32 = ops.linear(xd, wd, b, out_dtype=torch.float32, drop_p=0.1, seed=6, out_scale=0.5, residual=res)
            assert _rel(y8, y32) < 3e-5     # (the fp8 MFMA and the exact-f32 path round their sums differently)


@pytest.mark.parametrize("D", [256, 512, 1024])
def test_layernorm_fwd_mx_matches_quant_mx(D):
    """cfm_layernorm_fwd_mx: y, mean, rstd bit-identical to cfm_layernorm_fwd's bf16 forward, and its MX copy
    bit-identical to cfm_quant_mx of that y (ragged row count)."""
    g = torch.Generator().manual_seed(D)
    M = 1001
    x = (torch.randn(M, D, generator=g) * 3 + 1).to(DEV)
    gm = (1 + 0.1 * torch.randn(D, generator=g)).to(DEV)
    bt = (0.1 * torch.randn(D, generator=g)).to(DEV)
    y, (y8, s8), mu, rs = ops.layernorm_fwd_mx(x, gm, bt)
    y0, mu0, rs0 = ops.layernorm_fwd(x, gm, bt, out_dtype=torch.bfloat16)
    assert torch.equal(y, y0) and torch.equal(mu, mu0) and torch.equal(rs, rs0)
    q8, qs = ops.quant_mx(y0)
    assert torch.equal(s8, qs) and torch.equal(y8.view(torch.uint8), q8.view(torch.uint8))


def test_mx_gemm_ffn_up_mx_out():
    """The fp8 FFN-up launch's second output (cfm_gemm_desc.mx_out): the MX copy of its bf16 C is exactly quant_mx
    of that C, and C itself is unchanged by asking for it."""
    g = torch.Generator().manual_seed(9)
    M, N, K = 2999, 2048, 512
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (0.05 * torch.randn(N, K, generator=g)).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    xq, sx = ops.quant_mx(x)
    wq, sw = ops.quant_mx(w)
    pre0 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y0 = ops.linear(xq, wq, b, act=ops.ACT_SILU, pre=pre0, drop_p=0.1, seed=5, x_mx=sx, w_mx=sw)
    pre1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    h8 = torch.empty(M, N, device=DEV, dtype=torch.float8_e4m3fn)
    hs = torch.empty(M, N // 32, device=DEV, dtype=torch.uint8)
    y1 = ops.linear(xq, wq, b, act=ops.ACT_SILU, pre=pre1, drop_p=0.1, seed=5, x_mx=sx, w_mx=sw, mx_out=(h8, hs))
    assert torch.equal(y0, y1) and torch.equal(pre0, pre1)
    r8, rs = ops.quant_mx(y1)
    assert torch.equal(hs, rs) and torch.equal(h8.view(torch.uint8), r8.view(torch.uint8))
