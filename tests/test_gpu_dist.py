"""Data-parallel equality on the real hot path (SURVEY.md §4 test layer 4, §8e): two ranks (gloo,
both on cuda:0 -- the box has one GPU) each run the front-end + Conformer + CTC-head training step
on their half of a global batch, GradAllReducer averages the gradients (Conformer weight gradients
written straight into the flat buckets by the grouped launch, bucket all-reduces issued as each chunk
of layers is flushed); the averaged gradients must equal ONE process's gradients on the whole batch.
BatchNorm runs either on its running statistics (eval mode) or in train mode with cross-replica
statistics (Conformer.set_sync_batchnorm, the SyncBatchNorm split kernels): per-replica train-mode BN
statistics (DDP without SyncBN) would make the two sides legitimately differ.
Tolerance: relative L2 1e-4 per parameter (fp32 reduction-order differences only); 2e-2 for bf16 with
train-mode SyncBN (bf16 rounding flips of the normalised activations, the bf16 parity tolerance)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(cd, bn="eval"):
    sys.path.insert(0, REPO)
    import bench
    torch.manual_seed(0)
    m = bench.EncoderCTC(2, 144, 4, 576, 15, 40, 80, 201, 0.0, cd).cuda().train()
    if bn == "eval":
        m.conformers.eval()
    g = torch.Generator().manual_seed(5)
    x = torch.rand(4, 80, 201, generator=g).cuda()
    T2 = m.T2
    lens = torch.tensor([T2, T2 - 7, T2 - 20, T2], dtype=torch.int32).cuda()
    tgt = torch.randint(1, 40, (4, 9), generator=g).to(torch.int32).cuda()
    tl = torch.tensor([9, 5, 7, 3], dtype=torch.int32).cuda()
    return m, x, lens, tgt, tl


def _grads(m, x, lens, tgt, tl, reducer=None):
    loss, _ = m(x, lens, tgt, tl, seed=3)
    loss.backward()
    if reducer is not None:
        reducer.allreduce()
    torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}


def _step_fn(m, mb):
    def step():
        loss, _ = m(*mb, seed=3)
        loss.backward()
        return loss
    return step


def _graph_grads(m, mb, red):
    """One eager warm-up step (allocator, grouped-launch staging tables), then the step captured as a
    SegmentedStepGraph (cut at every chunk flush), replayed TWICE -- first on other inputs (x halved), then on
    the real ones -- with the buckets reduced after each replay: the result must be the second replay's
    gradients (a gradient copied into its bucket only once would stay at the first replay's values)."""
    from nn_conformer_for_speech_recognition_amd import dist as cdist
    _step_fn(m, mb)()
    red.allreduce()
    for p in m.parameters():
        p.grad = None
    seg = cdist.SegmentedStepGraph(red)
    seg.capture(_step_fn(m, mb))
    assert len(seg) >= 3                    # cut at the chunk flushes (chunk_layers=1: layers 1 and 0)
    x_real = mb[0].clone()
    mb[0].mul_(0.5)
    seg.replay()
    red.allreduce()
    mb[0].copy_(x_real)
    seg.replay()
    red.allreduce()
    torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}


def _worker(rank, world, port, cd, q, bn="eval", accum=False, mode="eager"):
    import faulthandler
    faulthandler.dump_traceback_later(100, exit=True)     # a stuck rank reports where, then exits
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    sys.path.insert(0, REPO)
    from nn_conformer_for_speech_recognition_amd import dist as cdist
    torch.cuda.set_device(0)
    cdist.init_from_env(backend="gloo")
    m, x, lens, tgt, tl = _setup(cd, bn)
    if bn == "sync":
        m.conformers.set_sync_batchnorm()
    if mode == "graph_unrouted":
        # a gradient hook on one weight keeps layer 0 out of the grouped launch: its gradients land in captured
        # pool tensors, not in the bucket views, and must be copied in again after every replay
        m.conformers.conformer_layers[0].ffn1.sequential[1].weight.register_hook(lambda g: g)
    red = cdist.GradAllReducer([p for p in m.parameters()], model=m, chunk_layers=1, overlap=True,
                               grad_dtype=torch.bfloat16 if mode == "graph_bf16" else torch.float32)
    sl = slice(2 * rank, 2 * rank + 2)
    mb = (x[sl].contiguous(), lens[sl].contiguous(), tgt[sl].contiguous(), tl[sl].contiguous())
    if accum:
        # gradient accumulation over two micro-batches (the same slice twice): the first backward runs under
        # no_sync (no bucket all-reduce), the second accumulates into the bucket views in place (no grouped
        # launch: .grad exists) and its chunks are reduced by allreduce(), never mid-backward
        with red.no_sync():
            loss, _ = m(*mb, seed=3)
            loss.backward()
        assert not red.launched
    g = _grads(m, *mb, red) if mode == "eager" else _graph_grads(m, mb, red)
    # the grouped gradients really are the bucket views (no copy-in)
    ok = None
    if m.conformers.grad_dest is not None:
        conf = m.conformers.conformer_layers[1]
        ok = conf.ffn1.sequential[1].weight.grad.data_ptr() == m.conformers.grad_dest[1][2][0].data_ptr()
    g.update({"buf." + n: b.detach().cpu().clone() for n, b in m.named_buffers() if "running" in n})
    q.put((rank, {n: t.numpy() for n, t in g.items()}, ok))    # by value (no shared-memory fds)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("cd,bn,accum,mode", [(torch.bfloat16, "eval", False, "eager"),
                                              (torch.float32, "eval", False, "eager"),
                                              (torch.bfloat16, "sync", False, "eager"),
                                              (torch.float32, "sync", False, "eager"),
                                              (torch.bfloat16, "eval", True, "eager"),
                                              (torch.float32, "eval", True, "eager"),
                                              (torch.bfloat16, "eval", False, "graph"),
                                              (torch.bfloat16, "eval", False, "graph_bf16"),
                                              (torch.bfloat16, "eval", False, "graph_unrouted")])
def test_two_rank_grads_equal_one_rank_full_batch(cd, bn, accum, mode):
    """bn='eval': BatchNorm on running statistics; bn='sync': train-mode BatchNorm with
    Conformer.set_sync_batchnorm() (cross-replica statistics) -- the running statistics must then
    also equal the single-process ones.  mode 'graph': the step as a SegmentedStepGraph (bucket reduces
    issued between segment replays); 'graph_bf16': the same with bf16 reduce copies of the buckets;
    'graph_unrouted': graph mode with one layer outside the grouped launch (gradient hook)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cd, q, bn, accum, mode)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = []
    for _ in range(240):                       # never block on a dead worker
        try:
            got.append(q.get(timeout=1))
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
        if len(got) == world:
            break
    assert len(got) == world
    out = sorted(got, key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m1, *data = _setup(cd, bn)
    if accum:                       # the single process accumulates the same two micro-batches
        loss, _ = m1(*data, seed=3)
        loss.backward()
    ref = _grads(m1, *data)
    ref.update({"buf." + n: b.detach().cpu().clone() for n, b in m1.named_buffers() if "running" in n})
    (_, g0, ok0), (_, g1, _) = out
    if cd == torch.bfloat16:
        assert ok0                  # (accum: the second micro-batch added in place into the bucket views)
    # train-mode BN in bf16: the replicas' fp32 partial sums are added in another order than the single
    # process's, which flips a few bf16 roundings of the normalised activations -> bf16-level noise
    tol = 2e-2 if (bn == "sync" and cd == torch.bfloat16) else 1e-4
    if mode == "graph_bf16":
        tol = 1e-2              # each rank's fp32 gradient rounded to bf16 before the sum
    for n, want in ref.items():
        a, b = torch.from_numpy(g0[n]).double(), torch.from_numpy(g1[n]).double()
        if bn == "sync" and n.endswith("conv_module.sequential.2.bias"):
            continue            # train-mode BN right after the depthwise conv: true gradient 0, both sides noise
        if n.startswith("buf."):                          # running statistics: local buffers, equal by SyncBN
            btol = 1e-5 if cd == torch.float32 else 1e-3
            assert ((a - want.double()).norm() / want.double().norm().clamp_min(1e-30)).item() < btol, n
            continue
        assert torch.equal(a, b), n                       # every rank holds the same averaged gradient
        err = ((a - want.double()).norm() / want.double().norm().clamp_min(1e-30)).item()
        assert err < tol, (n, err)


def test_segmented_graph_single_process_matches_eager():
    """World 1: the SegmentedStepGraph still cuts at every chunk flush (no reduce to issue); the chain of
    replays must give the eager backward's gradients, bit for bit, over two replays."""
    from nn_conformer_for_speech_recognition_amd import dist as cdist
    m, x, lens, tgt, tl = _setup(torch.bfloat16)
    mb = (x, lens, tgt, tl)
    red = cdist.GradAllReducer([p for p in m.parameters()], model=m, chunk_layers=1, overlap=True)
    ref = _grads(m, *mb, red)
    for p in m.parameters():
        p.grad = None
    seg = cdist.SegmentedStepGraph(red)
    seg.capture(_step_fn(m, mb))
    assert len(seg) == 3
    for _ in range(2):
        seg.replay()
        red.allreduce()
        torch.cuda.synchronize()
        got = {n: p.grad.detach().cpu() for n, p in m.named_parameters()}
        for n in ref:
            assert torch.equal(got[n], ref[n]), n
