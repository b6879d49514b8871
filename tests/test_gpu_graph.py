"""A whole training step (Conformer fwd + fused CTC head + bwd) captured into ONE HIP graph:
replays are bit-identical to eager steps at the same device dropout-counter value (cfm_rng_bind),
and successive replays draw different dropout masks.  Also the in-kernel timing probe."""
import pytest
import torch

from nn_conformer_for_speech_recognition_amd import _lib, ops
from nn_conformer_for_speech_recognition_amd.conformer import Conformer
from nn_conformer_for_speech_recognition_amd.ctc import ctc_head_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup():
    torch.manual_seed(0)
    B, T, d, V, U = 3, 40, 64, 24, 6
    model = Conformer(d, 2, 128, 2, 7, dropout=0.1).to(DEV).train()
    head = torch.nn.Linear(d, V).to(DEV)
    x = torch.randn(B * T, d, device=DEV)
    lens = torch.tensor([T, T - 7, 25], dtype=torch.int32, device=DEV)
    tgt = torch.randint(1, V, (B, U), dtype=torch.int32, device=DEV)
    tl = torch.tensor([U, 4, 3], dtype=torch.int32, device=DEV)
    return model, head, x, lens, tgt, tl, B, T


def test_graph_replay_matches_eager_and_redraws_dropout():
    model, head, x, lens, tgt, tl, B, T = _setup()
    params = list(model.parameters()) + list(head.parameters())
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    _lib.call("cfm_rng_bind", _lib.ptr(ctr))
    try:
        def step():
            ctr.add_(1)
            y = model.forward_tokens(x, lens, B, T, seed=5)
            loss, _ = ctc_head_loss(y, head.weight, head.bias, tgt, lens, tl, B, T, zero_infinity=True)
            loss.backward()
            return loss

        def grads():
            return torch.cat([p.grad.reshape(-1) for p in params]).clone()

        eager = []
        for _ in range(2):
            for p in params:
                p.grad = None
            eager.append((step().item(), grads()))
        assert eager[0][0] != eager[1][0]                  # counter 1 vs 2: different masks

        ctr.zero_()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):                      # warm-up outside the capture
            for p in params:
                p.grad = None
            step()
        torch.cuda.current_stream().wait_stream(side)
        for p in params:
            p.grad = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            static = step()
        for i, (want_loss, want_grad) in enumerate(eager):
            ctr.fill_(i)                                   # the captured add_(1) makes it i + 1
            g.replay()
            torch.cuda.synchronize()
            assert static.item() == want_loss
            assert torch.equal(grads(), want_grad)
    finally:
        _lib.call("cfm_rng_bind", None)


def test_probe_slot_times_a_gemm():
    M, N, K = 4096, 1024, 512
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    slot = torch.zeros(4, dtype=torch.int64, device=DEV)
    khz = _lib.load().cfm_wallclock_khz()
    assert khz > 0

    def probe(kind, shape, desc, launch):
        _lib.call("cfm_probe_slot", _lib.ptr(slot), 0, _lib.stream())
        desc.probe = _lib.ptr(slot)
        r = launch()
        _lib.call("cfm_probe_slot", _lib.ptr(slot), 1, _lib.stream())
        return r

    ops.PROBE = probe
    try:
        for _ in range(3):
            ops.linear(a, w, out=out)
    finally:
        ops.PROBE = None
    torch.cuda.synchronize()
    assert int(slot[3]) == 3
    us = int(slot[2]) / khz * 1e3 / 3
    assert 0.5 < us < 5000, us
    torch.testing.assert_close(out.float(), (a.float() @ w.float().T), rtol=2e-2, atol=2e-1)
