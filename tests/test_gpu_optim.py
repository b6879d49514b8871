"""libcfm Adafactor vs transformers.Adafactor (the reference's optimizer, runner.py:36) on the
same parameters and gradients, several steps, mixed tensor ranks (1-D, 2-D, 3-D, 4-D)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("beta1", [0.9, None])
def test_adafactor_matches_transformers(beta1, inplace):
    """inplace: gradients written into the same buffers every step (the captured-graph case) ->
    the host fast path that reuses the cached task table."""
    from transformers import Adafactor as HFAdafactor
    from nn_conformer_for_speech_recognition_amd.optim import Adafactor
    torch.manual_seed(0)
    shapes = [(37,), (64, 48), (16, 8, 3, 3), (24, 1, 7), (512, 256), (5,), (300, 2304), (2, 70, 100),
              (33, 3000)]
    ref = [torch.randn(s, dtype=torch.float64) for s in shapes]
    mine = [torch.nn.Parameter(r.float().cuda()) for r in ref]
    theirs = [torch.nn.Parameter(r.clone()) for r in ref]
    o1 = Adafactor(mine, lr=1e-2, beta1=beta1, scale_parameter=False, relative_step=False)
    o2 = HFAdafactor(theirs, lr=1e-2, beta1=beta1, scale_parameter=False, relative_step=False)
    for step in range(5):
        for a, b in zip(mine, theirs):
            g = torch.randn(a.shape, dtype=torch.float64) * (step + 1)
            if inplace and a.grad is not None:
                a.grad.copy_(g.float())
            else:
                a.grad = g.float().cuda()
            b.grad = g.clone()
        o1.step()
        o2.step()
    torch.cuda.synchronize()
    for a, b in zip(mine, theirs):
        err = (a.detach().double().cpu() - b.detach()).norm() / b.detach().norm()
        assert err < 1e-5, (tuple(a.shape), err.item())


def test_adafactor_relative_step():
    from transformers import Adafactor as HFAdafactor
    from nn_conformer_for_speech_recognition_amd.optim import Adafactor
    torch.manual_seed(1)
    a = torch.nn.Parameter(torch.randn(32, 16).cuda())
    b = torch.nn.Parameter(a.detach().cpu().double().clone())
    o1 = Adafactor([a], lr=None, scale_parameter=False, relative_step=True)
    o2 = HFAdafactor([b], lr=None, scale_parameter=False, relative_step=True)
    for _ in range(3):
        g = torch.randn(32, 16, dtype=torch.float64)
        a.grad, b.grad = g.float().cuda(), g.clone()
        o1.step()
        o2.step()
    assert ((a.detach().double().cpu() - b.detach()).norm() / b.detach().norm()) < 1e-5


def test_adafactor_load_state_dict_then_step():
    """Checkpoint resume: step, load a saved state dict (new state tensors), step again -- the cached
    device task table must follow the new state (it was keyed on param/grad pointers only)."""
    from transformers import Adafactor as HFAdafactor
    from nn_conformer_for_speech_recognition_amd.optim import Adafactor
    torch.manual_seed(2)
    shapes = [(64, 48), (37,), (8, 3, 5)]
    ref = [torch.randn(s, dtype=torch.float64) for s in shapes]
    mine = [torch.nn.Parameter(r.float().cuda()) for r in ref]
    theirs = [torch.nn.Parameter(r.clone()) for r in ref]
    o1 = Adafactor(mine, lr=1e-2, beta1=0.9, scale_parameter=False, relative_step=False)
    o2 = HFAdafactor(theirs, lr=1e-2, beta1=0.9, scale_parameter=False, relative_step=False)
    grads = [[torch.randn(s, dtype=torch.float64) for s in shapes] for _ in range(6)]

    def run(steps):
        for gs in steps:
            for a, b, g in zip(mine, theirs, gs):
                if a.grad is None:
                    a.grad = g.float().cuda()
                else:
                    a.grad.copy_(g.float())          # same buffers: the fast path would hit its cache
                b.grad = g.clone()
            o1.step()
            o2.step()

    run(grads[:2])
    import copy
    saved = copy.deepcopy(o1.state_dict())
    saved_hf = copy.deepcopy(o2.state_dict())
    run(grads[2:4])                                  # advance, then roll both optimizers back
    o1.load_state_dict(saved)
    o2.load_state_dict(saved_hf)
    run(grads[4:6])
    torch.cuda.synchronize()
    for a, b in zip(mine, theirs):
        err = (a.detach().double().cpu() - b.detach()).norm() / b.detach().norm()
        assert err < 1e-5, (tuple(a.shape), err.item())
