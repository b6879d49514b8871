"""Kernel-level parity on the GPU: each HIP kernel vs a plain PyTorch fp32 (CPU) reference of the
same op, and SpecAugment vs the oracle (bit-exact)."""
import json
import os
import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402

DEV = "cuda"


def _rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(257, 130, 77), (128, 128, 64), (1000, 512, 512), (33, 40, 1000)])
def test_gemm_layouts(dtype, ak, bk, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    ref = A @ B.T
    Ad = (A if ak else A.T.contiguous()).to(DEV, dtype)
    Bd = (B if bk else B.T.contiguous()).to(DEV, dtype)
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.gemm(Ad, Bd, C, M, N, K, a_kmajor=ak, b_kmajor=bk)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(C, ref) < tol


@pytest.fixture
def gemm_mode():
    from nn_conformer_for_speech_recognition_amd import _lib
    yield lambda m: _lib.call("cfm_gemm_set_mode", m)
    _lib.call("cfm_gemm_set_mode", 3)


# register-staged / LDS-DMA auto / 256x128 BK64 / BK32 / 192x128 (K-major x K-major: warp-specialised, 8 compute
# waves; + 524288: the shared-DMA 192-row pipeline) / 192x128 BK32 8 waves (AK only)
@pytest.mark.parametrize("mode", [1, 2, 18, 34, 82, 82 | 524288, 114])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(1000, 512, 512), (264, 136, 192), (520, 264, 1000), (8, 8, 64)])
def test_gemm_kernel_variants(gemm_mode, mode, ak, bk, M, N, K):
    """Every bf16 kernel variant (incl. the LDS-DMA pipeline's clamped M/N edges and zero-filled
    MN-major K tail) against an fp32 reference, bias + SiLU epilogue included."""
    gemm_mode(mode)
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + mode)
    A = torch.randn(M, K, generator=g).bfloat16().float()
    B = torch.randn(N, K, generator=g).bfloat16().float()
    bias = torch.randn(N, generator=g)
    z = A @ B.T + bias
    Ad = (A if ak else A.T.contiguous()).to(DEV, torch.bfloat16)
    Bd = (B if bk else B.T.contiguous()).to(DEV, torch.bfloat16)
    pre = torch.empty(M, N, device=DEV, dtype=torch.float32)
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm(Ad, Bd, C, M, N, K, a_kmajor=ak, b_kmajor=bk, bias=bias.to(DEV), act=ops.ACT_SILU, pre=pre)
    torch.cuda.synchronize()
    assert _rel(pre, z) < 1e-5
    assert _rel(C.float(), torch.nn.functional.silu(z)) < 1e-2


@pytest.mark.parametrize("mode", [1, 18, 34, 82])
def test_gemm_kernel_variants_splitk_batched(gemm_mode, mode):
    gemm_mode(mode)
    g = torch.Generator().manual_seed(17)
    M, N, K = 256, 192, 5000
    dy = torch.randn(K, M, generator=g).bfloat16().float()     # tokens x out  (MN-major operands)
    x = torch.randn(K, N, generator=g).bfloat16().float()
    for split in (1, 4, 8):
        dw = ops.linear_wgrad(dy.to(DEV, torch.bfloat16), x.to(DEV, torch.bfloat16), split_k=split)
        assert _rel(dw, dy.T @ x) < 1e-5
    # batched K-major x K-major with a batch stride (the attention-free batched form)
    Z, M2, N2, K2 = 3, 300, 136, 128
    A = torch.randn(Z, M2, K2, generator=g).bfloat16().float()
    B = torch.randn(Z, N2, K2, generator=g).bfloat16().float()
    C = torch.empty(Z, M2, N2, device=DEV)
    ops.gemm(A.to(DEV, torch.bfloat16), B.to(DEV, torch.bfloat16), C, M2, N2, K2, batch=Z,
             stride_a=M2 * K2, stride_b=N2 * K2, stride_c=M2 * N2)
    torch.cuda.synchronize()
    assert _rel(C, A @ B.transpose(1, 2)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dtype):
    g = torch.Generator().manual_seed(5)
    M, N, K = 300, 192, 96
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 0.1
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    pre = torch.empty(M, N, device=DEV, dtype=torch.float32)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.gemm(A.to(DEV, dtype), W.to(DEV, dtype), out, M, N, K, bias=bias.to(DEV), act=ops.ACT_SILU, pre=pre,
             out_scale=0.5, residual=res.to(DEV))
    z = A @ W.T + bias
    ref = 0.5 * torch.nn.functional.silu(z) + res
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(pre, z) < tol
    assert _rel(out, ref) < tol
    # act_grad epilogue: dgrad of silu
    dy = torch.randn(M, N, generator=g)
    dx = torch.empty(M, K, device=DEV, dtype=torch.float32)
    ops.linear_dgrad(dy.to(DEV, dtype), W.to(DEV, dtype), out=dx)
    assert _rel(dx, dy @ W) < tol
    dz = torch.empty(M, N, device=DEV, dtype=torch.float32)
    # (dy * silu'(pre)) via a GEMM epilogue: identity B
    eye = torch.eye(N)
    ops.gemm(dy.to(DEV, dtype), eye.to(DEV, dtype), dz, M, N, N, b_kmajor=True, act_grad=True, pre=pre)
    zr = z.requires_grad_()
    torch.nn.functional.silu(zr).backward(dy)
    assert _rel(dz, zr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("rows,cols", [(2048, 512), (512, 1536), (100, 70), (1, 64)])
def test_cast_transpose_batch(rows, cols):
    g = torch.Generator().manual_seed(rows + cols)
    srcs = [torch.randn(rows, cols, generator=g).to(DEV), torch.randn(cols, rows + 3, generator=g).to(DEV)]
    dsts = [torch.empty(t.shape[1], t.shape[0], device=DEV, dtype=torch.bfloat16) for t in srcs]
    plain = [torch.empty(t.shape, device=DEV, dtype=torch.bfloat16) for t in srcs]
    ops.CastTBatch(srcs, dsts).refresh()
    torch.cuda.synchronize()
    for s_, d_ in zip(srcs, dsts):
        assert torch.equal(d_, s_.t().to(torch.bfloat16))   # a cast + transpose: bit-exact
    dsts2 = [torch.empty_like(d_) for d_ in dsts]
    ops.CastTBatch(srcs, dsts2, plain).refresh()
    torch.cuda.synchronize()
    for s_, d_, p_ in zip(srcs, dsts2, plain):
        assert torch.equal(d_, s_.t().to(torch.bfloat16))
        assert torch.equal(p_, s_.to(torch.bfloat16))


def test_linear_dgrad_transposed_weight():
    """dX via the K-major W^T copy equals dX via the MN-major W path (same products, bf16)."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 1000, 2048, 512
    dy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.05).to(DEV)
    pre = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w16 = W.to(torch.bfloat16)
    wt = torch.empty(K, N, device=DEV, dtype=torch.bfloat16)
    ops.CastTBatch([W], [wt]).refresh()
    a = ops.linear_dgrad(dy, w16, out_dtype=torch.float32)
    b = ops.linear_dgrad(dy, w16, out_dtype=torch.float32, wt=wt)
    ref = dy.float() @ w16.float()
    assert _rel(a, ref) < 1e-5 and _rel(b, ref) < 1e-5
    a = ops.linear_dgrad(dy[:, :K], w16[:K, :K].contiguous(), pre=pre, act_grad=True, drop_p=0.1, seed=4)
    b = ops.linear_dgrad(dy[:, :K], w16[:K, :K].contiguous(), pre=pre, act_grad=True, drop_p=0.1, seed=4,
                         wt=w16[:K, :K].t().contiguous())
    assert _rel(a.float(), b.float()) < 1e-2
    assert torch.equal(a == 0, b == 0)   # identical dropout masks


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_wgrad_splitk(dtype):
    g = torch.Generator().manual_seed(9)
    M, N, K = 5000, 256, 144
    dy = torch.randn(M, N, generator=g)
    x = torch.randn(M, K, generator=g)
    for split in (1, 8):
        dw = ops.linear_wgrad(dy.to(DEV, dtype), x.to(DEV, dtype), split_k=split)
        assert _rel(dw, dy.T @ x) < (1e-5 if dtype == torch.float32 else 1e-2)


def test_gemm_dropout_deterministic():
    M, N, K = 256, 256, 64
    A = torch.randn(M, K, device=DEV)
    W = torch.randn(N, K, device=DEV)
    o1 = torch.empty(M, N, device=DEV)
    o2 = torch.empty(M, N, device=DEV)
    ops.gemm(A, W, o1, M, N, K, drop_p=0.25, seed=11, offset=3)
    ops.gemm(A, W, o2, M, N, K, drop_p=0.25, seed=11, offset=3)
    assert torch.equal(o1, o2)
    frac = (o1 == 0).float().mean().item()
    assert 0.2 < frac < 0.3
    ref = A @ W.T
    kept = o1 != 0
    assert torch.allclose(o1[kept], ref[kept] / 0.75, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("D", [144, 256, 512, 100, 64, 200, 384])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm(D, dtype):
    """64 * V widths on the one-row-per-wave kernels, other multiples of 8 (Conformer-S 144, 64, 200, 384) on the
    lane-group kernels, the rest (100) on the generic strided kernels."""
    g = torch.Generator().manual_seed(D)
    M = 777
    x = torch.randn(M, D, generator=g) * 2 + 0.3
    gamma = torch.rand(D, generator=g) + 0.5
    beta = torch.randn(D, generator=g)
    y, mean, rstd = ops.layernorm_fwd(x.to(DEV), gamma.to(DEV), beta.to(DEV), out_dtype=dtype)
    xr = x.clone().requires_grad_()
    gr = gamma.clone().requires_grad_()
    br = beta.clone().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-5)
    assert _rel(y, yr) < (1e-6 if dtype == torch.float32 else 5e-3)
    dy = torch.randn(M, D, generator=g)
    dres = torch.randn(M, D, generator=g)
    yr.backward(dy)
    dx, dgamma, dbeta = ops.layernorm_bwd(dy.to(DEV, dtype), x.to(DEV), gamma.to(DEV), mean, rstd,
                                          dres=dres.to(DEV))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(dx, xr.grad + dres) < tol
    assert _rel(dgamma, gr.grad) < tol
    assert _rel(dbeta, br.grad) < tol


def test_specaug_bit_exact_vs_oracle(golden_dir):
    from oracle import specaug as osa
    from nn_conformer_for_speech_recognition_amd import specaugment as psa
    with open(os.path.join(golden_dir, "specaug.json")) as f:
        cases = json.load(f)
    for c in cases:
        hp = SimpleNamespace(warping_param_W=c["W"], warping_ntimes=c["warping_ntimes"],
                             frequency_mask_param_F=c["F_param"], frequency_mask_ntimes=c["frequency_mask_ntimes"],
                             time_multiplicity=c["time_multiplicity"],
                             adaptive_multiplicity=c["adaptive_multiplicity"], pm=c["pm"], ps=c["ps"],
                             adaptive_size=c["adaptive_size"], time_mask_param_T=c["T_param"], mask_value=0)
        x = np.array(c["x"], np.float32)
        for mode in ("reference", "intended"):
            random.seed(c["seed"])
            d = osa.draw(c["B"], c["F"], c["tau"], hp)
            ref = osa.apply(x, c["tau"], d, mode=mode)
            random.seed(c["seed"])
            y = psa.spec_augment(torch.tensor(x, device=DEV), c["tau"], hp, intended=(mode == "intended"))
            np.testing.assert_array_equal(y.cpu().numpy(), ref)
        np.testing.assert_array_equal(ref if False else osa.apply(x, c["tau"], d, "reference"),
                                      np.array(c["y"], np.float32))


def test_specaug_large_bit_exact():
    from oracle import specaug as osa
    from nn_conformer_for_speech_recognition_amd import specaugment as psa
    from nn_conformer_for_speech_recognition_amd.lib.hparams import HParams
    hp = HParams(None)
    B, F, T = 32, 80, 1501
    g = torch.Generator().manual_seed(0)
    x = torch.rand(B, F, T, generator=g)
    tau = [T - 13 * i for i in range(B)]
    random.seed(42)
    d = osa.draw(B, F, tau, hp)
    ref = osa.apply(x.numpy(), tau, d, mode="intended")
    random.seed(42)
    y = psa.spec_augment(x.to(DEV), tau, hp, intended=True)
    np.testing.assert_array_equal(y.cpu().numpy(), ref)


@pytest.mark.parametrize("B,F,T", [(2, 80, 201), (1, 9, 7), (3, 16, 100)])
def test_conv1_mfma_fwd_and_wgrad(B, F, T):
    """conv1 (1 -> 512 ch, 7x7, stride 2) on the matrix cores (bf16 NHWC output, x as hi+lo bf16):
    forward within bf16 output rounding of the fp32 conv, weight/bias gradients of a bf16 dh1
    within 1e-4 of the fp32 reduction of the same dh1."""
    g = torch.Generator().manual_seed(B * 1000 + T)
    x = torch.rand(B, F, T, generator=g)
    w = torch.randn(512, 49, generator=g) * 0.2
    b = torch.randn(512, generator=g)
    h1 = ops.conv1_fwd(x.to(DEV), w.to(DEV), b.to(DEV), torch.bfloat16)
    ref = torch.nn.functional.conv2d(x.unsqueeze(1), w.view(512, 1, 7, 7), b, stride=2)   # (B, 512, F1, T1)
    ref = ref.permute(0, 2, 3, 1)
    assert h1.shape == ref.shape
    assert _rel(h1.float(), ref) < 4e-3
    w16 = w.to(torch.bfloat16).float()
    ref16 = torch.nn.functional.conv2d(x.unsqueeze(1), w16.view(512, 1, 7, 7), b, stride=2).permute(0, 2, 3, 1)
    assert (h1.float().cpu() - ref16).abs().max().item() <= 1e-2 * ref16.abs().max().item()
    dh1 = torch.randn(ref.shape, generator=g).to(torch.bfloat16)
    dw, db = ops.conv1_bwd_weight(dh1.to(DEV), x.to(DEV), 512)
    xr = x.unsqueeze(1).double().requires_grad_()
    wr = w.view(512, 1, 7, 7).double().requires_grad_()
    br = b.double().requires_grad_()
    torch.nn.functional.conv2d(xr, wr, br, stride=2).backward(dh1.double().permute(0, 3, 1, 2))
    assert _rel(dw, wr.grad.view(512, 49)) < 1e-4
    assert _rel(db, br.grad) < 1e-5


@pytest.mark.parametrize("B,F1,T1,C1,C2", [(2, 37, 100, 512, 128), (1, 9, 11, 64, 32), (2, 10, 8, 128, 64)])
def test_conv2_bwd_data_pipeline(gemm_mode, B, F1, T1, C1, C2):
    """conv2 data-gradient on the LDS-DMA pipeline (gathered dh2 rows, packed per-class weights)
    against the transposed convolution in fp64, and against the register-staged gather path."""
    g = torch.Generator().manual_seed(F1 * T1 + C1)
    F2, T2 = (F1 - 3) // 2 + 1, (T1 - 3) // 2 + 1
    W = (torch.randn(C2, C1, 3, 3, generator=g) * 0.05).to(torch.bfloat16)
    dh2 = torch.randn(B, T2, F2, C2, generator=g).to(torch.bfloat16)
    w2r = W.permute(0, 2, 3, 1).reshape(C2, 9 * C1).contiguous()
    ref = torch.nn.functional.conv_transpose2d(dh2.double().permute(0, 3, 2, 1), W.double(), stride=2,
                                               output_padding=(F1 - (2 * F2 + 1), T1 - (2 * T2 + 1)))
    ref = ref.permute(0, 2, 3, 1)          # (B, F1, T1, C1)
    fast = ops.conv2_bwd_data(dh2.to(DEV), w2r.to(DEV), F1, T1)
    gemm_mode(1)                           # no LDS-DMA pipeline: the register-staged gather kernel
    slow = ops.conv2_bwd_data(dh2.to(DEV), w2r.to(DEV), F1, T1)
    torch.cuda.synchronize()
    assert fast.shape == ref.shape
    assert _rel(fast.float(), ref) < 1e-2
    assert _rel(fast.float(), slow.float()) < 1e-2


@pytest.mark.parametrize("B,F1,T1,C1,C2", [(2, 37, 100, 512, 128), (1, 9, 11, 64, 32), (2, 10, 8, 128, 64)])
def test_conv2_fwd_pipeline(gemm_mode, B, F1, T1, C1, C2):
    """conv2 forward (3x3, stride 2) as the LDS-DMA implicit GEMM with h1 rows gathered per tap,
    against conv2d in fp64 and against the register-staged implicit GEMM."""
    g = torch.Generator().manual_seed(F1 + T1 * C2)
    W = (torch.randn(C2, C1, 3, 3, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(C2, generator=g)
    h1 = torch.randn(B, F1, T1, C1, generator=g).to(torch.bfloat16)
    w2r = W.permute(0, 2, 3, 1).reshape(C2, 9 * C1).contiguous()
    ref = torch.nn.functional.conv2d(h1.double().permute(0, 3, 1, 2), W.double(), bias.double(), stride=2)
    ref = ref.permute(0, 3, 2, 1)         # (B, T2, F2, C2)
    fast = ops.conv2_fwd(h1.to(DEV), w2r.to(DEV), bias.to(DEV), torch.float32)
    gemm_mode(1)
    slow = ops.conv2_fwd(h1.to(DEV), w2r.to(DEV), bias.to(DEV), torch.float32)
    torch.cuda.synchronize()
    assert fast.shape == ref.shape
    assert _rel(fast, ref) < 1e-5
    assert _rel(fast, slow) < 1e-5


@pytest.mark.parametrize("D", [512, 144, 200, 100])
def test_layernorm_bwd_fused_dropout_output(D):
    """cfm_layernorm_bwd_drop's g2 is bit-identical to cfm_scale_dropout(dx) (fused for D = 512 and the lane-group
    widths 144 / 200, the separate pass for 100), dx unchanged."""
    g = torch.Generator().manual_seed(D)
    M = 1000
    x = torch.randn(M, D, generator=g).to(DEV)
    gamma = torch.randn(D, generator=g).to(DEV)
    beta = torch.randn(D, generator=g).to(DEV)
    _, mu, rs = ops.layernorm_fwd(x, gamma, beta, out_dtype=torch.bfloat16)
    dy = torch.randn(M, D, generator=g).to(DEV, torch.bfloat16)
    dres = torch.randn(M, D, generator=g).to(DEV)
    dx0, gg0, gb0 = ops.layernorm_bwd(dy, x, gamma, mu, rs, dres=dres)
    dx1, gg1, gb1, g2 = ops.layernorm_bwd(dy, x, gamma, mu, rs, dres=dres, drop=(0.5, 0.1, 77, torch.bfloat16))
    ref = ops.scale_dropout(dx0, 0.5, 0.1, 77, 0, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1) and torch.equal(gg0, gg1) and torch.equal(gb0, gb1)
    assert torch.equal(g2, ref)


@pytest.mark.parametrize("M,N,K,split", [(5000, 256, 144, 8), (11936, 2048, 512, None), (3000, 512, 512, 1),
                                         (2000, 1536, 512, 4)])
def test_wgrad_fused_bias_grad(M, N, K, split):
    """linear_wgrad(bias_out=): the bias gradient sum_rows(dy) from the weight-gradient GEMM's staged dy
    tiles + split-K reduction (cfm_gemm_desc.a_colsum), or cfm_colsum when split-K is off."""
    g = torch.Generator().manual_seed(M + N)
    dy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    db = torch.empty(N, device=DEV)
    dw = ops.linear_wgrad(dy, x, split_k=split, bias_out=db)
    torch.cuda.synchronize()
    assert _rel(db, dy.double().sum(0)) < 1e-5
    assert _rel(dw, dy.double().t() @ x.double()) < 1e-5


def test_wgrad_group_matches_per_gemm():
    """cfm_wgrad_group (one launch, whole token reduction per tile) against fp64 dyᵀ x and sum_rows dy."""
    g = torch.Generator().manual_seed(8)
    M = 1500
    shapes = [(2048, 512), (512, 2048), (1536, 512), (512, 512), (1024, 512), (136, 72)]
    grp = ops.WgradGroup()
    outs, refs = [], []
    for N, K in shapes:
        dy = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
        x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
        outs.append(grp.add(dy, x))
        refs.append((dy.double().t() @ x.double(), dy.double().sum(0)))
    grp.flush()
    torch.cuda.synchronize()
    for (dw, db), (rw, rb) in zip(outs, refs):
        assert _rel(dw, rw) < 1e-5
        assert _rel(db, rb) < 1e-5


def test_wgrad_group_planned_l15_matches_unplanned():
    """The planned grouped launch (cfm_wgrad_group_plan: whole-task rounds per XCD, the ragged last round's 28
    tiles split over 8 K slices + the slab reduction) at the L15 backward's exact task list (17 layers x 8 GEMMs,
    M 11,936) against the unplanned launch: unsplit tasks bit-identical (same tiles, same k order), split tasks
    within fp32 summation-order noise; the split tasks against fp32 references too."""
    M, d, F = 32 * 373, 512, 2048
    g = torch.Generator(device=DEV).manual_seed(3)
    shapes = [(d, F), (F, d), (d, d), (2 * d, d), (d, d), (3 * d, d), (d, F), (F, d)]   # backward order, per layer
    pairs = [(torch.randn(M, n, device=DEV, generator=g).to(torch.bfloat16),
              torch.randn(M, k, device=DEV, generator=g).to(torch.bfloat16)) for _ in range(17) for n, k in shapes]
    res = {}
    try:
        for plan in (False, True):
            ops.WGRAD_PLAN = plan
            grp = ops.WgradGroup()
            res[plan] = [grp.add(dy, x) for dy, x in pairs]
            grp.flush()
            torch.cuda.synchronize()
    finally:
        ops.WGRAD_PLAN = True
    lib = _lib.load()
    tiles = np.array([lib.cfm_wgrad_group_tiles(dy.shape[1], x.shape[1]) for dy, x in pairs], dtype=np.int64)
    cap = int(tiles.sum()) * 16 + 512
    sched, split = np.empty(cap, dtype=np.uint32), np.zeros(len(pairs), dtype=np.int32)
    assert lib.cfm_wgrad_group_plan(tiles.ctypes.data, len(pairs), 8, 32, sched.ctypes.data, cap, split.ctypes.data) > 0
    assert (split > 1).sum() == 7
    for i, ((w0, b0), (w1, b1)) in enumerate(zip(res[False], res[True])):
        if split[i] == 1:
            assert torch.equal(w0, w1) and torch.equal(b0, b1), i
        else:
            assert _rel(w1, w0) < 1e-6 and _rel(b1, b0) < 1e-6, i
            dy, x = pairs[i]
            assert _rel(w1, dy.float().T @ x.float()) < 1e-5
            assert _rel(b1, dy.float().sum(0)) < 1e-5


@pytest.mark.parametrize("M", [1000, 11936, 37])
def test_wgrad_group_wide_tiles_vs_reference(M):
    """The grouped weight-gradient launch (256 x 256 shared-DMA tiles) on the encoder's shapes, incl. the fused bias
    gradient, ragged N / K and a token count that is not a multiple of the 32-deep step, against fp32 references."""
    g = torch.Generator().manual_seed(11 + M)
    shapes = [(2048, 512), (512, 2048), (1536, 512), (512, 512), (136, 264)]
    ops_ = [(torch.randn(M, N, generator=g).to(DEV, torch.bfloat16), torch.randn(M, K, generator=g).to(DEV, torch.bfloat16))
            for N, K in shapes]
    grp = ops.WgradGroup()
    res = [grp.add(d, x) for d, x in ops_]
    grp.flush()
    torch.cuda.synchronize()
    for (a, ab), (d, x) in zip(res, ops_):
        ref = d.float().T @ x.float()
        assert _rel(a, ref) < 1e-5
        assert _rel(ab, d.float().sum(0)) < 1e-5


@pytest.mark.parametrize("M,K", [(11936, 2048), (11936, 512), (1000, 1536), (385, 1024), (192, 64)])
@pytest.mark.parametrize("epi", ["bf16", "residual_drop", "rowdot", "batched"])
def test_gemm_warp_specialised_matches_shared_dma(gemm_mode, M, K, epi):
    """The warp-specialised d-wide kernel (default for K-major x K-major GEMMs with <= 512 output columns) against
    the shared-DMA 192-row pipeline (cfm_gemm_set_mode bit 19): the same 16x16x32 MFMAs in
    the same k order and the same epilogue -> bit-identical outputs (ragged M, every epilogue the encoder uses:
    bf16 data gradients, fp32 residual-stream forwards with dropout + 0.5 scale, the rowdot of attention's D,
    batched overlapping-row operands as the front-end fold uses)."""
    N = 512
    g = torch.Generator().manual_seed(M + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    with_ = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    T = M // 8 if M % 8 == 0 else M
    outs = []
    for mode in (3, 3 | 524288):
        gemm_mode(mode)
        if epi == "bf16":
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(x, w, y, M, N, K)
            outs.append((y.clone(),))
        elif epi == "residual_drop":
            y = torch.empty(M, N, device=DEV, dtype=torch.float32)
            ops.linear(x, w, b, out=y, drop_p=0.1, seed=7, out_scale=0.5, residual=res)
            outs.append((y.clone(),))
        elif epi == "rowdot":
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            D = torch.empty(M * N // 64, device=DEV, dtype=torch.float32)
            ops.gemm(x, w, y, M, N, K, rowdot=(with_, D, T))
            outs.append((y.clone(), D.clone()))
        else:
            # 4 batches of overlapping A rows (lda < K) as the folded front-end's windowed view
            Bb, Mb, lda = 4, M // 4, max(64, K // 2)
            y = torch.empty(Bb * Mb, N, device=DEV, dtype=torch.float32)
            ops.gemm(x, w, y, Mb, N, K, lda=lda, stride_a=Mb * lda, batch=Bb, stride_c=Mb * N, bias=b,
                     allow_overlap=True)
            outs.append((y.clone(),))
    torch.cuda.synchronize()
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("M", [11936, 4100])
@pytest.mark.parametrize("N", [1024, 1536, 640])
def test_gemm_wide_ws_matches_pipe(gemm_mode, M, N):
    """1024- / 1536-wide K-major x K-major outputs (QKV, pointwise-conv-1 forward) run on the warp-specialised kernel;
    cfm_gemm_set_mode bit 21 keeps the two-per-CU 192-row pipeline.  Same 16x16x32 MFMAs in the same k order and the
    same epilogue kinds -> bit-identical (bias-only and SiLU + pre-activation + dropout rows, ragged M)."""
    K = 512
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    outs = []
    for mode in (3, 3 | 2097152):
        gemm_mode(mode)
        y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.linear(x, w, b, out=y)
        ys = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.linear(x, w, b, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=9, out=ys)
        outs.append((y.clone(), ys.clone(), pre.clone()))
    torch.cuda.synchronize()
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    assert _rel(outs[0][0].float(), x.float() @ w.float().T + b) < 1e-2


@pytest.mark.parametrize("M", [11936, 1000, 385])
@pytest.mark.parametrize("epi,N", [("silu_pre_drop", 2048), ("actg_drop", 2048), ("bias", 1536), ("bias", 1024),
                                   ("f32_bias", 2048), ("res_drop", 512), ("res_drop", 2048), ("rowdot", 512),
                                   ("plain", 512), ("silu_pre_drop", 512)])
def test_gemm_fast_epilogue_matches_generic(gemm_mode, M, epi, N):
    """The compile-time epilogue kinds (epi_rows_fast: inputs issued ahead of the stores, bias loaded once) against
    the generic per-row epilogue_store8 path (cfm_gemm_set_mode bit 14) on the same kernels: the same arithmetic in
    the same order -> bit-identical outputs, for every kind the encoder launches, on the 256-row two-per-CU tiles
    (2048 wide), the 192-row tiles (1024 / 1536) and the warp-specialised d-wide kernel (512), ragged M."""
    K = 512
    g = torch.Generator().manual_seed(M + N + len(epi))
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    pre_in = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    with_ = torch.randn(M, N, generator=g).to(DEV, torch.bfloat16)
    T = M // 8 if M % 8 == 0 else M
    outs = []
    for mode in (3, 3 | 16384):
        gemm_mode(mode)
        if epi == "silu_pre_drop":
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.linear(x, w, b, act=ops.ACT_SILU, pre=pre, drop_p=0.1, seed=5, out=y)
            outs.append((y.clone(), pre.clone()))
        elif epi == "actg_drop":
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(x, w, y, M, N, K, pre=pre_in, act_grad=True, drop_p=0.1, seed=6)
            outs.append((y.clone(),))
        elif epi == "bias":
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.linear(x, w, b, out=y)
            outs.append((y.clone(),))
        elif epi == "f32_bias":
            y = torch.empty(M, N, device=DEV, dtype=torch.float32)
            ops.linear(x, w, b, out=y, out_scale=0.5)
            outs.append((y.clone(),))
        elif epi == "res_drop":
            y = torch.empty(M, N, device=DEV, dtype=torch.float32)
            ops.linear(x, w, b, out=y, drop_p=0.1, seed=7, out_scale=0.5, residual=res)
            outs.append((y.clone(),))
        elif epi == "rowdot":
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            D = torch.empty(M * N // 64, device=DEV, dtype=torch.float32)
            ops.gemm(x, w, y, M, N, K, rowdot=(with_, D, T))
            outs.append((y.clone(), D.clone()))
        else:
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(x, w, y, M, N, K)
            outs.append((y.clone(),))
    torch.cuda.synchronize()
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    if epi == "silu_pre_drop":   # and the values themselves (fp32 reference of the same epilogue)
        pre_ref = (x.float() @ w.float().T + b)
        assert _rel(outs[0][1].float(), pre_ref) < 1e-2
        kept = outs[0][0] != 0
        assert 0.87 < kept.float().mean().item() < 0.93
        act = torch.nn.functional.silu(pre_ref) / 0.9
        assert _rel(outs[0][0].float()[kept], act[kept]) < 1e-2


@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("sync", [False, True])
@pytest.mark.parametrize("B,T,C,K,dt", [(2, 37, 64, 31, torch.bfloat16), (3, 100, 96, 3, torch.float32),
                                        (1, 129, 200, 33, torch.bfloat16), (2, 64, 512, 15, torch.bfloat16),
                                        (2, 50, 66, 31, torch.bfloat16)])
def test_bn_folded_dwconv_bwd(training, sync, B, T, C, K, dt):
    """cfm_glu_dwconv_bwd_bn (BatchNorm1d + SiLU input gradient formed inside the depthwise backward) vs a
    torch fp64 autograd reference of GLU -> depthwise conv -> BatchNorm1d -> SiLU, and vs the unfused
    bn_silu_bwd + glu_dwconv_bwd pair.  sync: the SyncBatchNorm route with an identity all-reduce."""
    if sync and not training:
        pytest.skip("SyncBatchNorm backward is a training-mode path")
    g = torch.Generator().manual_seed(B * 1000 + T + C + K)
    a = torch.randn(B * T, 2 * C, generator=g)
    w = torch.randn(C, K, generator=g) * 0.3
    bias = torch.randn(C, generator=g) * 0.1
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    dz = torch.randn(B * T, C, generator=g)
    rm, rv = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5

    # reference (fp64, CPU autograd)
    ad = a.double().requires_grad_()
    wd, bd = w.double().requires_grad_(), bias.double().requires_grad_()
    gd, btd = gamma.double().requires_grad_(), beta.double().requires_grad_()
    u = torch.nn.functional.glu(ad.view(B, T, 2 * C), dim=-1).transpose(1, 2)
    y = torch.nn.functional.conv1d(u, wd.view(C, 1, K), bd, padding=(K - 1) // 2, groups=C)
    if training:
        mu, var = y.mean(dim=(0, 2)), y.var(dim=(0, 2), unbiased=False)
    else:
        mu, var = rm.double(), rv.double()
    yh = (y - mu[None, :, None]) / torch.sqrt(var[None, :, None] + 1e-5)
    z = torch.nn.functional.silu(yh * gd[None, :, None] + btd[None, :, None])
    (z.transpose(1, 2).reshape(B * T, C) * dz.double()).sum().backward()

    ad_, wd_, bd_ = a.to(DEV, dt), w.to(DEV), bias.to(DEV)
    gam, bet = gamma.to(DEV), beta.to(DEV)
    ws = ops.convmod_ws(B, T, C, K, DEV)
    yv = ops.glu_dwconv_fwd(ad_, wd_, bd_, B, T, C, K, ws)
    _, mean, invstd = ops.bn_silu_fwd(yv, gam, bet, rm.to(DEV), rv.to(DEV), 0.1, 1e-5, training, B, T, C, ws, dt)
    dzd = dz.to(DEV, dt)
    red = (lambda t: None) if sync else None
    da, dw, db, dg, dbt = ops.bn_silu_glu_dwconv_bwd(dzd, yv, gam, bet, mean, invstd, training, ad_, wd_, B, T, C,
                                                     K, ws, dt, reduce_sums=red, world=1)
    dy, dg2, dbt2 = ops.bn_silu_bwd(dzd, yv, gam, bet, mean, invstd, training, ws)
    da2, dw2, db2 = ops.glu_dwconv_bwd(dy, ad_, wd_, B, T, C, K, ws, dt)
    torch.cuda.synchronize()
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    assert _rel(da.float(), ad.grad) < tol
    assert _rel(dw, wd.grad) < tol
    if training:    # batch-stat BN cancels the depthwise bias: its true gradient is 0, ours is rounding noise
        assert (db.double().cpu() - bd.grad).norm() < tol * wd.grad.norm()
    else:
        assert _rel(db, bd.grad) < tol
    assert _rel(dg, gd.grad) < tol and _rel(dbt, btd.grad) < tol
    # same formula, same summation order as the unfused pair
    assert _rel(da.float(), da2.float()) < 1e-5
    assert _rel(dw, dw2) < 1e-5 and (db - db2).norm() < 1e-5 * dw.norm()
    assert torch.equal(dg, dg2) and torch.equal(dbt, dbt2)

@pytest.mark.parametrize("M,N,K", [(11936, 144, 144), (11936, 576, 144), (11936, 432, 144), (11936, 144, 432),
                                   (11936, 144, 288), (1000, 512, 8), (777, 2048, 72), (500, 144, 576),
                                   (3000, 1024, 200)])
def test_gemm_k_tail_pipeline(gemm_mode, M, N, K):
    """K-major GEMMs whose K is a multiple of 8 but not of the 64-deep tile (Conformer-S: K 144 / 288 / 432) on the
    LDS-DMA pipeline and the warp-specialised kernel: the last K tile's chunks past K read zero (out-of-range DMA
    offsets) instead of the next row's head.  fp32 output and the fp32 residual-stream epilogue against fp64 of the
    bf16 operands, and against the register-staged kernel (cfm_gemm_set_mode 1)."""
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.1).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV)
    ref = x.double() @ w.double().T
    outs = {}
    for mode in (3, 1):
        gemm_mode(mode)
        y = torch.empty(M, N, device=DEV, dtype=torch.float32)
        ops.gemm(x, w, y, M, N, K)
        yr = torch.empty(M, N, device=DEV, dtype=torch.float32)
        ops.linear(x, w, b, out=yr, out_scale=0.5, residual=res)
        yb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.gemm(x, w, yb, M, N, K)
        torch.cuda.synchronize()
        outs[mode] = (y, yr, yb)
    for mode, (y, yr, yb) in outs.items():
        assert _rel(y, ref) < 1e-5, mode
        assert _rel(yr, res.double() + 0.5 * (ref + b.double())) < 1e-5, mode
        assert _rel(yb.float(), ref) < 5e-3, mode
    assert _rel(outs[3][0], outs[1][0]) < 1e-5


@pytest.mark.parametrize("D", [512, 144, 256, 100])
def test_layernorm_bf16_residual_input(D):
    """LayerNorm forward / backward reading a bf16 x (the bf16 mode's residual stream inside a layer, conformer.py
    RES_BF16): against torch on the same bf16 values in fp32; the MX forward (fp8 mode) bit-identical to quant_mx of
    its bf16 y."""
    g = torch.Generator().manual_seed(D + 3)
    M = 555
    x = (torch.randn(M, D, generator=g) * 2 + 0.3).to(torch.bfloat16)
    gamma = torch.rand(D, generator=g) + 0.5
    beta = torch.randn(D, generator=g)
    y, mean, rstd = ops.layernorm_fwd(x.to(DEV), gamma.to(DEV), beta.to(DEV), out_dtype=torch.bfloat16)
    xr = x.float().clone().requires_grad_()
    gr, br = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-5)
    assert _rel(y, yr) < 5e-3
    dy = torch.randn(M, D, generator=g).to(torch.bfloat16)
    dres = torch.randn(M, D, generator=g)
    yr.backward(dy.float())
    dx, dgamma, dbeta = ops.layernorm_bwd(dy.to(DEV), x.to(DEV), gamma.to(DEV), mean, rstd, dres=dres.to(DEV))
    assert dx.dtype == torch.float32
    assert _rel(dx, xr.grad + dres) < 1e-5
    assert _rel(dgamma, gr.grad) < 1e-5 and _rel(dbeta, br.grad) < 1e-5
    if D in (256, 512):
        y2, (y8, s8), _, _ = ops.layernorm_fwd_mx(x.to(DEV), gamma.to(DEV), beta.to(DEV))
        q8, qs = ops.quant_mx(y2)
        torch.cuda.synchronize()
        assert torch.equal(y2, y) and torch.equal(y8.view(torch.uint8), q8.view(torch.uint8)) and torch.equal(s8, qs)


@pytest.mark.parametrize("res_dt,out_dt", [(torch.bfloat16, torch.bfloat16), (torch.float32, torch.bfloat16),
                                           (torch.float32, torch.float32)])
@pytest.mark.parametrize("M,N,K", [(11936, 512, 2048), (11936, 512, 512), (3000, 144, 576), (777, 256, 1024)])
def test_gemm_residual_epilogue_dtypes(gemm_mode, res_dt, out_dt, M, N, K):
    """The residual-add epilogue kinds (EF_F32_RES, EF_BF16_RES, EF_F32R_BF16): out = residual + out_scale *
    dropout(x·wᵀ + b), bit-identical to the generic epilogue rows (cfm_gemm_set_mode bit 14) on the same main loop,
    and within rounding of fp64."""
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    res = torch.randn(M, N, generator=g).to(DEV, res_dt)
    outs = []
    for mode in (3, 3 | 16384):
        gemm_mode(mode)
        y = torch.empty(M, N, device=DEV, dtype=out_dt)
        ops.linear(x, w, b, out=y, drop_p=0.1, seed=11, out_scale=0.5, residual=res)
        outs.append(y.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    y0 = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.linear(x, w, b, out=y0, out_scale=0.5, residual=res.float())   # no dropout: the fp64 check
    ref = res.double() + 0.5 * (x.double() @ w.double().T + b.double())
    assert _rel(y0, ref) < 1e-5


@pytest.mark.parametrize("M,N,K", [(11936, 512, 2048), (11936, 512, 512), (3000, 144, 576), (11936, 256, 1024),
                                   (777, 2048, 512)])
@pytest.mark.parametrize("drop_p,out_scale", [(0.1, 0.5), (0.1, 1.0), (0.0, 0.5)])
def test_gemm_delta_epilogue(gemm_mode, M, N, K, drop_p, out_scale):
    """The residual module's output without the residual (EF_BF16_DELTA: bf16 out_scale * dropout(x·wᵀ + b), the
    RES_FUSE form whose add the next LayerNorm does): bit-identical to the generic epilogue rows (cfm_gemm_set_mode
    bit 14) on the same main loop, and equal to the fp32 residual epilogue's output minus its residual up to the
    bf16 rounding of the delta (same dropout mask)."""
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    outs = []
    for mode in (3, 3 | 16384):
        gemm_mode(mode)
        y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.linear(x, w, b, out=y, drop_p=drop_p, seed=11, out_scale=out_scale)
        outs.append(y.clone())
    gemm_mode(3)
    zero = torch.zeros(M, N, device=DEV)
    yr = torch.empty(M, N, device=DEV)
    ops.linear(x, w, b, out=yr, drop_p=drop_p, seed=11, out_scale=out_scale, residual=zero)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], yr.to(torch.bfloat16))


@pytest.mark.parametrize("D", [512, 256, 144, 1024, 128, 100])
@pytest.mark.parametrize("dd", [torch.bfloat16, torch.float32])
def test_layernorm_fwd_residual_add(D, dd):
    """cfm_layernorm_fwd_res: x' = x + delta (fp32, exactly the fp32 sum) and y = LN(x') -- bit-identical to
    cfm_layernorm_fwd of x' (the same kernel family on the same values); with the MX copy (fp8 mode, D in 256 / 512 /
    1024) bit-identical to layernorm_fwd_mx of x'; ragged M (555 rows, a partial last workgroup)."""
    g = torch.Generator().manual_seed(D + 11)
    M = 555
    x = (torch.randn(M, D, generator=g) * 2 + 0.3).to(DEV)
    delta = torch.randn(M, D, generator=g).to(DEV, dd)
    gamma = (torch.rand(D, generator=g) + 0.5).to(DEV)
    beta = torch.randn(D, generator=g).to(DEV)
    for od in (torch.bfloat16, torch.float32):
        xo, y, mean, rstd = ops.layernorm_fwd_res(x, delta, gamma, beta, out_dtype=od)
        xs = x + delta.float()
        y2, mean2, rstd2 = ops.layernorm_fwd(xs, gamma, beta, out_dtype=od)
        torch.cuda.synchronize()
        assert torch.equal(xo, xs)
        if (dd == torch.bfloat16 and D % 64 == 0) or D == 100:   # the vector kernels, the generic kernel
            assert torch.equal(y, y2) and torch.equal(mean, mean2) and torch.equal(rstd, rstd2)
        else:   # an fp32 delta takes the generic kernel (another summation order than the vector kernels); the lane-
            # group kernel (D 144) differs from its plain instantiation in the last bit of rstd (contraction choices)
            assert _rel(y, y2) < (5e-3 if od == torch.bfloat16 else 1e-5) and _rel(rstd, rstd2) < 1e-6
            assert _rel(mean, mean2) < 1e-6
    if D in (256, 512, 1024) and dd == torch.bfloat16:
        xo, y, (y8, s8), mean, rstd = ops.layernorm_fwd_res(x, delta, gamma, beta, mx=True)
        ym, (q8, qs), _, _ = ops.layernorm_fwd_mx(x + delta.float(), gamma, beta)
        torch.cuda.synchronize()
        assert torch.equal(y, ym) and torch.equal(y8.view(torch.uint8), q8.view(torch.uint8)) and torch.equal(s8, qs)


@pytest.mark.parametrize("M,K", [(11936, 1024), (11936, 256), (1000, 768)])
@pytest.mark.parametrize("res", [False, True])
def test_gemm_ws96_narrow_outputs(gemm_mode, M, K, res):
    """256-wide outputs (Conformer-M's d) on the 96-row warp-specialised tiles (250 tiles at M 11,936 where 192-row
    tiles give 126) against the 192-row warp-specialised kernel (cfm_gemm_set_mode bit 23): the same 16x16x32 MFMAs
    in the same k order and the same epilogue -> bit-identical, bf16 data-gradient and fp32 residual epilogues."""
    N = 256
    g = torch.Generator().manual_seed(M + K + res)
    x = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    r = torch.randn(M, N, generator=g).to(DEV)
    outs = []
    for mode in (3, 3 | 8388608):
        gemm_mode(mode)
        if res:
            y = torch.empty(M, N, device=DEV, dtype=torch.float32)
            ops.linear(x, w, b, out=y, drop_p=0.1, seed=5, out_scale=0.5, residual=r)
        else:
            y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(x, w, y, M, N, K)
        outs.append(y.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    if not res:
        assert _rel(outs[0].float(), x.double() @ w.double().T) < 5e-3
