"""BiLSTM decoder on libcfm vs the reference's own op, torch.nn.LSTM.

The reference (asrnn.py:38,252) runs nn.LSTM(256, 512, bidirectional=True) on the 2-D encoder output:
one unbatched sequence of L = B*T_enc steps.  The checker is torch.nn.LSTM on the CPU in float64 with the
same weights (the reference's op at higher precision).  Tolerances (fp32 recurrence vs fp64): output and
h_n relative L2 <= 2e-5 and per-row max-abs <= 1e-4; gradients relative L2 <= 2e-4."""
import pytest
import torch

from nn_conformer_for_speech_recognition_amd.lstm import LSTM

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _pair(In, H, layers, bidir, seed):
    torch.manual_seed(seed)
    ref = torch.nn.LSTM(In, H, num_layers=layers, bidirectional=bidir).double()
    mine = LSTM(In, H, num_layers=layers, bidirectional=bidir).to(DEV)
    mine.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    return ref, mine


@pytest.mark.parametrize("L,In,H,layers,bidir", [
    (1, 256, 512, 1, True),          # single step (no recurrence term, no dW_hh)
    (7, 40, 32, 1, False),           # small, unidirectional
    (300, 256, 512, 1, True),        # the reference decoder's dims
    (1280, 256, 512, 1, True),       # the reference's native shape: B 32 x 40 frames
    (200, 64, 128, 2, True),         # stacked layers (eval-style: no inter-layer dropout)
])
def test_lstm_fwd_bwd_vs_torch(L, In, H, layers, bidir):
    ref, mine = _pair(In, H, layers, bidir, seed=L + H)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(L, In, generator=g, dtype=torch.float64)
    dy = torch.randn(L, H * (2 if bidir else 1), generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr, (hr, cr) = ref(xr)
    (yr * dy).sum().backward()

    xm = x.float().to(DEV).requires_grad_(True)
    ym, (hm, cm) = mine(xm)
    (ym * dy.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()

    assert ym.shape == yr.shape and hm.shape == hr.shape and cm.shape == cr.shape
    assert _rel(ym, yr) < 2e-5
    assert (ym.double().cpu() - yr.detach()).abs().amax().item() < 1e-4
    assert _rel(hm, hr) < 2e-5 and _rel(cm, cr) < 2e-5
    assert _rel(xm.grad, xr.grad) < 2e-4
    pr = dict(ref.named_parameters())
    for name, p in mine.named_parameters():
        assert _rel(p.grad, pr[name].grad) < 2e-4, name
    LSTM.check_errors()      # the recurrences' wait-limit flags (kept on the device, no per-launch sync)


def test_lstm_long_sequence_direction_symmetry():
    """Size-independent property at a long L (the L15 decoder's 11,936 steps): running the reverse
    direction on the time-flipped input equals a unidirectional LSTM with the reverse weights."""
    L, In, H = 11936, 256, 512
    torch.manual_seed(3)
    bi = LSTM(In, H, bidirectional=True).to(DEV)
    uni = LSTM(In, H, bidirectional=False).to(DEV)
    with torch.no_grad():
        uni.weight_ih_l0.copy_(bi.weight_ih_l0_reverse)
        uni.weight_hh_l0.copy_(bi.weight_hh_l0_reverse)
        uni.bias_ih_l0.copy_(bi.bias_ih_l0_reverse)
        uni.bias_hh_l0.copy_(bi.bias_hh_l0_reverse)
    x = torch.randn(L, In, device=DEV)
    y_bi, _ = bi(x)
    y_uni, _ = uni(x.flip(0))
    assert (y_bi[:, H:] - y_uni.flip(0)).abs().amax().item() < 1e-5
    assert torch.isfinite(y_bi).all()
    LSTM.check_errors()


def test_lstm_no_host_sync_per_layer():
    """The forward / backward issue no blocking device read (a per-layer .item() stalled the host
    queue): with torch's sync debug mode set to error, a 2-layer bidirectional pass runs through."""
    torch.manual_seed(5)
    m = LSTM(64, 128, num_layers=2, bidirectional=True).to(DEV)
    x = torch.randn(50, 64, device=DEV, requires_grad=True)
    m(x)        # first call: lazily allocates the flag word and its pinned host copy
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        y, _ = m(x)
        y.sum().backward()
    finally:
        torch.cuda.set_sync_debug_mode(0)
    LSTM.check_errors()
    assert torch.isfinite(x.grad).all()


def test_lstm_state_dict_matches_torch_names():
    a = torch.nn.LSTM(256, 512, bidirectional=True).state_dict()
    b = LSTM(256, 512, bidirectional=True).state_dict()
    assert list(a) == list(b) and all(a[k].shape == b[k].shape for k in a)
