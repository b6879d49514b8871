"""The folded 'frame'-mode front-end (frontfold.hip: ConvSubSampling -> per-frame Linear -> dropout as ONE
GEMM over a strided view of the packed mels) against the unfolded composition it replaces
(lib/convsubsampling.py:41-43 conv_sub_1 -> conv_sub_2, then the standard_linear of asrnn.py:208 per frame)
computed in fp64 by torch on the CPU, and against the unfolded libcfm kernels (CFM_FFOLD=0).

Tolerances (relative L2): fp32 operands 2e-6 forward / 2e-5 gradients (fp32 sums in a different order);
bf16 with the hi + lo split of x 4e-3 / 1e-2 (the folded weight and the dropout-scaled output gradient
are rounded to bf16 once); bf16 hi only 1e-2 / 1.5e-2."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from nn_conformer_for_speech_recognition_amd import frontend as fe  # noqa: E402
from nn_conformer_for_speech_recognition_amd.lib.convsubsampling import ConvSubSampling  # noqa: E402
from nn_conformer_for_speech_recognition_amd.lib.hparams import HParams  # noqa: E402

DEV = "cuda"


def rel_err(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def make(B, Fb, T, C1, C2, D, seed=0):
    torch.manual_seed(seed)
    hp = HParams(None)
    hp.conv_sub_1_nodes = C1
    hp.set_input_dim(Fb, T)
    cs = ConvSubSampling(hp, 1, C2)
    F1, T1 = (Fb - 7) // 2 + 1, (T - 7) // 2 + 1
    F2, T2 = (F1 - 3) // 2 + 1, (T1 - 3) // 2 + 1
    proj = torch.nn.Linear(F2 * C2, D)
    with torch.no_grad():   # non-trivial biases (nn.Conv2d's init is small)
        for m in (cs.conv_sub_1, cs.conv_sub_2, proj):
            m.bias.uniform_(-0.5, 0.5)
    x = torch.rand(B, Fb, T)
    return cs, proj, x, (F2, T2)


def reference(cs, proj, x, gy):
    """fp64 CPU: conv2d -> conv2d -> (B, T2, F2*C2) frames -> Linear; grads of all six parameters."""
    ps = [p.detach().double().clone().requires_grad_() for p in
          (cs.conv_sub_1.weight, cs.conv_sub_1.bias, cs.conv_sub_2.weight, cs.conv_sub_2.bias, proj.weight, proj.bias)]
    h = F.conv2d(x.double().unsqueeze(1), ps[0], ps[1], stride=2)
    h = F.conv2d(h, ps[2], ps[3], stride=2)                       # (B, C2, F2, T2)
    B, C2, F2, T2 = h.shape
    fr = h.permute(0, 3, 2, 1).reshape(B * T2, F2 * C2)           # features (f2, c2)
    y = F.linear(fr, ps[4], ps[5])
    y.backward(gy.double())
    return y.detach(), [p.grad for p in ps]


def run_fold(cs, proj, x, gy, cd, drop_p=0.0, seed=5, hilo=True, fold=True):
    cs = cs.to(DEV)
    proj = proj.to(DEV)
    for p in list(cs.parameters()) + list(proj.parameters()):
        p.grad = None
    old = os.environ.get("CFM_FFOLD")
    os.environ["CFM_FFOLD"] = "1" if fold else "0"
    try:
        y = fe.frame_frontend(cs, proj, x.to(DEV), cd, drop_p=drop_p, seed=seed, hilo=hilo)
        y.backward(gy.to(DEV))
    finally:
        if old is None:
            del os.environ["CFM_FFOLD"]
        else:
            os.environ["CFM_FFOLD"] = old
    torch.cuda.synchronize()
    grads = [p.grad.detach().cpu() for p in (cs.conv_sub_1.weight, cs.conv_sub_1.bias, cs.conv_sub_2.weight,
                                             cs.conv_sub_2.bias, proj.weight, proj.bias)]
    return y.detach().cpu(), grads


NAMES = ("conv_sub_1.weight", "conv_sub_1.bias", "conv_sub_2.weight", "conv_sub_2.bias", "proj.weight", "proj.bias")
SHAPES = [(2, 80, 161, 512, 128, 144), (3, 80, 301, 64, 32, 256), (1, 64, 97, 72, 16, 64), (2, 83, 150, 40, 24, 96)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", ["fp32", "bf16_hilo", "bf16_hi"])
def test_fold_vs_fp64_composition(shape, mode):
    cs, proj, x, (F2, T2) = make(*shape)
    B, D = shape[0], shape[5]
    gy = torch.randn(B * T2, D)
    ref, rgrads = reference(cs, proj, x, gy)
    cd = torch.float32 if mode == "fp32" else torch.bfloat16
    y, grads = run_fold(cs, proj, x, gy, cd, hilo=(mode != "bf16_hi"))
    tol_y, tol_g = {"fp32": (2e-6, 2e-5), "bf16_hilo": (4e-3, 1e-2), "bf16_hi": (1e-2, 1.5e-2)}[mode]
    assert y.shape == ref.shape
    assert rel_err(y, ref) < tol_y
    for n, g, r in zip(NAMES, grads, rgrads):
        assert g.shape == r.shape, n
        assert rel_err(g, r) < tol_g, (n, rel_err(g, r))


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16])
def test_fold_dropout_matches_unfolded_kernels(cd):
    """Same dropout masks as the unfolded projection GEMM's epilogue (element index (b T2 + t2) D + o)."""
    cs, proj, x, (F2, T2) = make(2, 80, 201, 128, 32, 128, seed=3)
    gy = torch.randn(2 * T2, 128)
    y1, g1 = run_fold(cs, proj, x, gy, cd, drop_p=0.2, seed=77)
    y0, g0 = run_fold(cs, proj, x, gy, cd, drop_p=0.2, seed=77, fold=False)
    assert torch.equal(y1 == 0, y0 == 0)       # identical masks
    assert (y1 == 0).float().mean().item() > 0.1
    tol = 1e-5 if cd == torch.float32 else 2e-2
    assert rel_err(y1, y0) < tol
    for n, a, b in zip(NAMES, g1, g0):
        assert rel_err(a, b) < (1e-4 if cd == torch.float32 else 3e-2), n


def test_fold_conformer_L_shape_and_determinism():
    """BASELINE configs[1] front-end (32 x 80 x 1501, 512 / 128 channels, D 512): bf16 fold vs the fp32 fold,
    finite, and bit-identical on a second run (no atomics)."""
    cs, proj, x, (F2, T2) = make(32, 80, 1501, 512, 128, 512, seed=1)
    assert (F2, T2) == (18, 373)
    gy = torch.randn(32 * T2, 512) * 1e-2
    y32, g32 = run_fold(cs, proj, x, gy, torch.float32, drop_p=0.1, seed=9)
    yb, gb = run_fold(cs, proj, x, gy, torch.bfloat16, drop_p=0.1, seed=9)
    yb2, gb2 = run_fold(cs, proj, x, gy, torch.bfloat16, drop_p=0.1, seed=9)
    assert torch.isfinite(yb).all() and all(torch.isfinite(g).all() for g in gb)
    assert rel_err(yb, y32) < 4e-3
    for n, a, b in zip(NAMES, gb, g32):
        assert rel_err(a, b) < 1e-2, n
    assert torch.equal(yb, yb2) and all(torch.equal(a, b) for a, b in zip(gb, gb2))


def test_fold_graph_replay():
    """The fold (pack, compose, GEMM, backward contractions) captured in a HIP graph replays bit-identically."""
    cs, proj, x, (F2, T2) = make(4, 80, 301, 256, 64, 128, seed=2)
    cs, proj = cs.to(DEV), proj.to(DEV)
    xd = x.to(DEV)
    gy = torch.randn(4 * T2, 128, device=DEV)
    params = list(cs.parameters()) + list(proj.parameters())

    def step():
        for p in params:
            p.grad = None
        y = fe.frame_frontend(cs, proj, xd, torch.bfloat16, drop_p=0.1, seed=4)
        y.backward(gy)
        return y

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y_e = step().clone()
        g_e = [p.grad.clone() for p in params]
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    for p in params:
        p.grad = None
    with torch.cuda.graph(graph):
        y_g = step()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(y_g, y_e)
    for p, g in zip(params, g_e):
        assert torch.equal(p.grad, g)
