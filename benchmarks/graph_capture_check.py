"""tests/test_gpu_graph.py's capture with toggles: python graph_repro2.py [wt|nowt|norefresh]"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nn_conformer_for_speech_recognition_amd import _lib, ops  # noqa: E402
from nn_conformer_for_speech_recognition_amd import conformer as cm  # noqa: E402
from nn_conformer_for_speech_recognition_amd.ctc import ctc_head_loss  # noqa: E402

mode = sys.argv[1]
if mode in ("nowt", "norefresh"):
    cm._wt = lambda cfg, i: None
if mode == "norefresh":
    ops.CastTBatch.refresh = lambda self: None
if mode == "notable":
    cm._wt = lambda cfg, i: None

    class _NoT:
        def __init__(self, srcs, dsts):
            pass

        def refresh(self):
            pass
    ops.CastTBatch = _NoT
torch.manual_seed(0)
B, T, d, V, U = 3, 40, 64, 24, 6
model = cm.Conformer(d, 2, 128, 2, 7, dropout=0.1).to("cuda").train()
head = torch.nn.Linear(d, V).to("cuda")
x = torch.randn(B * T, d, device="cuda")
lens = torch.tensor([T, T - 7, 25], dtype=torch.int32, device="cuda")
tgt = torch.randint(1, V, (B, U), dtype=torch.int32, device="cuda")
tl = torch.tensor([U, 4, 3], dtype=torch.int32, device="cuda")
params = list(model.parameters()) + list(head.parameters())
ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
_lib.call("cfm_rng_bind", _lib.ptr(ctr))


def step():
    ctr.add_(1)
    y = model.forward_tokens(x, lens, B, T, seed=5)
    loss, _ = ctc_head_loss(y, head.weight, head.bias, tgt, lens, tl, B, T, zero_infinity=True)
    loss.backward()
    return loss


for _ in range(int(os.environ.get("NEAGER", "2"))):
    for p in params:
        p.grad = None
    step()
print(mode, "eager ok", flush=True)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for p in params:
        p.grad = None
    step()
torch.cuda.current_stream().wait_stream(side)
for p in params:
    p.grad = None
print(mode, "capturing", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    static = step()
g.replay()
torch.cuda.synchronize()
print(mode, "ok", static.item(), flush=True)
_lib.call("cfm_rng_bind", None)
