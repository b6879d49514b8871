"""Throughput benchmark: mel-frames/s of the Conformer-L encoder training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config L15]
    (N > 1: either under python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N, or plain
    `python bench.py --gpus N`, which starts that launcher itself as a child process; --gpus must equal the
    launcher's WORLD_SIZE, else the run exits 2)

One step = one utterance batch through the hot path, forward + backward:
ConvSubSampling -> frame projection -> 17 Conformer-L layers -> fused CTC head (Linear d->V +
log_softmax + CTC loss, ctc.hip) -> full backward -> (N>1) RCCL gradient all-reduce -> Adafactor
step.  Forward + backward are captured once into a HIP graph and replayed (--eager: launched from
Python every step); dropout masks still change every step (device step counter, cfm_rng_bind).  Inputs are synthetic 80-bin log-mel batches already resident in HBM
(SURVEY.md §8d), weights random-init.  Weak scaling: B=32 utterances per GPU.

Prints ONE JSON line (rank 0) with the contract fields plus `roofline` (dominant kernel, measured
live with HIP events on its launch stream over the timed region) and `cpu_baseline` (the CPU
oracle, rank 0 at N=1 only, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from nn_conformer_for_speech_recognition_amd import _lib  # noqa: E402
from nn_conformer_for_speech_recognition_amd import dist as cdist  # noqa: E402
from nn_conformer_for_speech_recognition_amd import ops  # noqa: E402
from nn_conformer_for_speech_recognition_amd import specaugment  # noqa: E402
from nn_conformer_for_speech_recognition_amd.ctc import ctc_head_loss, set_nonfinite_counter  # noqa: E402
from nn_conformer_for_speech_recognition_amd.conformer import Conformer  # noqa: E402
from nn_conformer_for_speech_recognition_amd.frontend import frame_frontend, linear  # noqa: E402
from nn_conformer_for_speech_recognition_amd.lib.convsubsampling import ConvSubSampling  # noqa: E402
from nn_conformer_for_speech_recognition_amd.lib.hparams import HParams  # noqa: E402
from nn_conformer_for_speech_recognition_amd.optim import Adafactor  # noqa: E402

METRIC = "mel-frames/sec/GPU Conformer-L encoder fwd+bwd; 1/2/4/8-GPU scaling"
# (name, layers, d, heads, ffn, K, batch per GPU, seconds, positional encoding) -- BASELINE.json configs:
# S15 = configs[1], M15 = configs[2] (run with --specaug), L15 = the metric's model at configs[1]'s shape
# (the headline line), L60 = configs[4] (60 s long-form, relative-position attention)
CONFIGS = {
    "L15": ("Conformer-L", 17, 512, 8, 2048, 31, 32, 15, "none"),
    "M15": ("Conformer-M", 16, 256, 4, 1024, 31, 32, 15, "none"),
    "S15": ("Conformer-S", 16, 144, 4, 576, 31, 32, 15, "none"),
    "L60": ("Conformer-L", 17, 512, 8, 2048, 31, 8, 60, "rel"),
}
PEAK_BF16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA
PEAK_FP8_TFLOPS = 5000.0      # MI355X_MICROARCH.md:44: ~5 PF dense fp8 (block-scaled e4m3 MFMA: 2x the bf16 rate)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def algorithmic_flops_per_frame(L, d, H, ffn, K, T_in, T2, F2, C1=512, C2=128, rel=False, B=1):
    """per-layer per-encoder-frame MACs 4*d*ffn + 4d^2 + 3d^2 + K*d + 2*T*d
    (+ T*d + (2T-1)*d^2/(B*T) with relative positions: the bd scores and linear_pos), the
    front-end (conv1 + conv2 + frame projection), x2 FLOPs, fwd+bwd = 3x fwd minus conv1's dgrad."""
    F1, T1 = (80 - 7) // 2 + 1, (T_in - 7) // 2 + 1
    per = 4 * d * ffn + 7 * d * d + K * d + 2 * T2 * d
    if rel:
        per += T2 * d + (2 * T2 - 1) * d * d / (B * T2)
    enc = L * T2 * per
    conv1 = C1 * 49 * F1 * T1
    conv2 = C2 * C1 * 9 * F2 * T2
    proj = T2 * F2 * C2 * d
    fwd = 2 * (enc + conv1 + conv2 + proj)
    fwdbwd = 3 * fwd - 2 * conv1
    return fwd / T_in, fwdbwd / T_in


def executed_flops_per_frame(L, d, H, ffn, K, T_in, T2, rel=False, B=1, Kp=1792, T2p=None):
    """The FLOPs the step EXECUTES per mel frame (fwd+bwd), for step_executed_tflops / step_mfma_frac: the
    encoder as in algorithmic_flops_per_frame, but the front-end as the folded GEMMs that replace conv1 + conv2 +
    projection: the forward GEMM 2*T2*Kp*d and the weight-gradient GEMM 2*T2p*Kp*d per utterance
    (Kp = 11 frames x 80 mels x hi+lo, padded; no input gradient); the fold's ~1 GFLOP/step of fp32 weight
    contractions is not counted.  The CTC head is excluded (reported separately)."""
    per = 4 * d * ffn + 7 * d * d + K * d + 2 * T2 * d
    if rel:
        per += T2 * d + (2 * T2 - 1) * d * d / (B * T2)
    enc = L * T2 * per
    T2p = T2 + 2 if T2p is None else T2p
    front = 2 * T2 * Kp * d + 2 * T2p * Kp * d
    return (3 * 2 * enc + front) / T_in


class EncoderCTC(torch.nn.Module):
    """Front-end + Conformer encoder + CTC head (the hot path of SURVEY.md §8a, 'frame' mode)."""

    def __init__(self, L, d, H, ffn, K, V, F_bins, T_in, dropout, cd, pos_enc="none", fp8=False):
        super().__init__()
        hp = HParams(None)
        hp.set_input_dim(F_bins, T_in)
        self.hp = hp
        self.cd = cd
        self.conv_sub_sampling = ConvSubSampling(hp, 1, hp.conv_sub_2_nodes)
        self.F1, self.T1 = (F_bins - 7) // 2 + 1, (T_in - 7) // 2 + 1
        self.F2, self.T2 = (self.F1 - 3) // 2 + 1, (self.T1 - 3) // 2 + 1
        self.standard_linear = torch.nn.Linear(self.F2 * hp.conv_sub_2_nodes, d)
        self.conformers = Conformer(d, H, ffn, L, K, dropout, pos_enc=pos_enc, compute_dtype=cd, fp8=fp8)
        self.ctc_fc = torch.nn.Linear(d, V)
        self.dropout = dropout

    def forward(self, x, lens_i32, targets_i32, tgt_lens_i32, seed, specaug_params=None):
        """-> (CTC loss (mean, zero_infinity), logits (B, T2, V)).  The head is the fused
        Linear + log_softmax + CTC node (ctc.hip); dropout seeds are offset on the device by the
        bound step counter, so one captured graph replays with fresh masks.  specaug_params: the
        device parameter block of this step's SpecAugment draws (specaugment.pack) -- the warp +
        masks then run as the first kernel of the step (asrnn.py:196-197)."""
        B = x.shape[0]
        if specaug_params is not None:
            x = specaugment.apply(x, specaug_params, intended=True)
        p = self.dropout if self.training else 0.0
        h = frame_frontend(self.conv_sub_sampling, self.standard_linear, x, self.cd, drop_p=p, seed=seed)
        y = self.conformers.forward_tokens(h, lens_i32, B, self.T2, seed=seed + 7)
        return ctc_head_loss(y, self.ctc_fc.weight, self.ctc_fc.bias, targets_i32, lens_i32, tgt_lens_i32, B,
                             self.T2, blank=0, reduction="mean", zero_infinity=True, compute_dtype=self.cd)


def run_nst(args, model, x, lens_i32, dev, cfg, rank, world):
    """BASELINE.json configs[3]: the NST pseudo-label pass (runner.py:253-281) -- eval-mode front-end +
    Conformer-L encoder (BatchNorm running stats, no dropout) + CTC head logits + device greedy decode
    with <pad>/<blank> stripped on the device (cfm_ctc_greedy_decode), one HIP graph per batch.  Weak
    scaling: each rank labels its own shard of B utterances; the label lists would be all-gathered once
    per pass (Runner.generate_labels), outside the per-batch loop timed here."""
    from nn_conformer_for_speech_recognition_amd.ctc import greedy_decode
    name, L, d, H, ffn, K, B, secs, pos_enc = cfg
    T_in = x.shape[-1]
    model.eval()

    def label_pass():
        with torch.no_grad():
            h = frame_frontend(model.conv_sub_sampling, model.standard_linear, x, model.cd)
            y = model.conformers.forward_tokens(h, lens_i32, B, model.T2, seed=1)
            logits = linear(y, model.ctc_fc.weight, model.ctc_fc.bias, cd=model.cd).view(B, model.T2, -1)
            return greedy_decode(logits, lens_i32, blank=0, pad=-1, collapse=False)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(max(args.warmup, 1)):
            label_pass()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = label_pass()
    graph.replay()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        graph.replay()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = tt.item()
    fwd_pf, _ = algorithmic_flops_per_frame(L, d, H, ffn, K, T_in, model.T2, model.F2, rel=pos_enc == "rel", B=B)
    ms = 1000.0 * elapsed / args.steps
    value = B * T_in * world * args.steps / elapsed
    res = {"metric": "mel-frames/sec/GPU Conformer-L NST pseudo-label pass (eval fwd + greedy CTC decode)",
           "value": round(value, 1), "unit": "mel-frames/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "bf16", "data": "synthetic (uniform min-max-normalised 80-bin mels, random init)",
           "config": {"workload": f"BASELINE configs[3]: {name} NST label pass, {B} x {secs} s utterances per GPU",
                      "model": name, "layers": L, "d_model": d, "pos_enc": pos_enc, "global_batch": B * world,
                      "seq_len": T_in, "enc_frames": model.T2, "parallelism": f"dp{world} (sharded utterances)",
                      "launch": "hip-graph (fwd + decode)"},
           "per_gpu_value": round(value / world, 1),
           "dist_backend": torch.distributed.get_backend() if torch.distributed.is_initialized() else None,
           "world_size_reported": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
           "step_algorithmic_tflops": round(fwd_pf * B * T_in / (ms * 1e-3) / 1e12, 1),
           "labels_nonempty": int((out[2] > 0).sum().item())}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


_ELT = {_lib.F32: 4, _lib.BF16: 2, _lib.FP8: 1}


def gemm_desc_bytes(desc):
    """Algorithmic HBM bytes of one cfm_gemm launch from its descriptor: A (M x K per batch) and B (N x K, per batch
    when strided) read in dtype_ab, C (M x N per batch) written in dtype_c, the residual (M x N) read in dtype_r --
    the definition benchmarks/pmc_dgemm_json.py uses for the PMC record's `algorithmic_bytes_per_launch`."""
    bt = max(1, int(desc.batch))
    ea, ec = _ELT[int(desc.dtype_ab)], _ELT[int(desc.dtype_c)]
    b_batches = bt if desc.stride_b else 1
    n = ea * (desc.M * desc.K * bt + desc.N * desc.K * b_batches) + ec * desc.M * desc.N * bt
    if desc.residual:
        n += _ELT[int(desc.dtype_r)] * desc.M * desc.N * bt
    if desc.mx_a:      # MX fp8: the e8m0 block scales of A and B (one byte per 32 K-elements of a row)
        n += (desc.M * bt + desc.N * b_batches) * (desc.K // 32)
    if desc.mx_out:    # the FFN-up epilogue's MX e4m3 copy of its output (+ its block scales)
        n += desc.M * desc.N * bt + desc.M * (desc.N // 32) * bt
    return float(n)


class KernelProbe:
    """Timing of one kernel family, installed as ops.PROBE.  Each matching launch gets a probe slot
    (cfm_gemm_desc.probe, 8 x u64): a one-lane kernel on the same stream resets the slot and stamps the wall clock
    right before the launch (cfm_probe_slot mode 2), the kernel itself records its first workgroup's start and its
    last workgroup's end (s_memrealtime), and a one-lane kernel after it stamps again and accumulates (mode 3):
    * `busy` = first-workgroup start -> last-workgroup end (the launch's own execution);
    * `incl` = stamp -> stamp around the launch MINUS the same interval of empty stamp pairs (calibrate(): the
      two one-lane kernels alone), i.e. the time the launch adds to a serial stream -- its dispatch ramp,
      execution and end-of-kernel completion, what rocprofv3's kernel trace counts; `frac` uses it.
    Works eagerly and inside a captured HIP graph (every replay accumulates)."""

    MAX_SLOTS = 1024
    CAL_PAIRS = 32

    def __init__(self, match, device):
        self.match = match
        self.active = False
        self.slots = torch.zeros(self.MAX_SLOTS, 8, dtype=torch.int64, device=device)
        self.cal = torch.zeros(self.CAL_PAIRS, 8, dtype=torch.int64, device=device)
        self.used = 0
        self.khz = _lib.load().cfm_wallclock_khz()
        self.slot_flops = [0.0] * self.MAX_SLOTS    # 2*M*N*K*batch of the launch each slot times (GEMMs)
        self.slot_bytes = [0.0] * self.MAX_SLOTS    # gemm_desc_bytes of that launch

    def __call__(self, kind, shape, desc, launch):
        if not (self.active and self.match(kind, shape, desc)) or self.khz <= 0:
            return launch()
        slot = self.used % self.MAX_SLOTS
        self.used += 1
        if kind == "gemm":
            M, N, K = shape
            self.slot_flops[slot] = 2.0 * M * N * K * max(1, int(desc.batch))
            self.slot_bytes[slot] = gemm_desc_bytes(desc)
        ptr = _lib.ptr(self.slots[slot])
        _lib.call("cfm_probe_slot", ptr, 2, _lib.stream())
        desc.probe = ptr
        r = launch()
        desc.probe = None
        _lib.call("cfm_probe_slot", ptr, 3, _lib.stream())
        return r

    def calibrate(self):
        """CAL_PAIRS empty (stamp, accumulate) pairs on the current stream -- launched inside the probe graph's
        capture, so every replay re-measures the one-lane kernels' own interval."""
        if self.khz <= 0:
            return
        for i in range(self.CAL_PAIRS):
            ptr = _lib.ptr(self.cal[i])
            _lib.call("cfm_probe_slot", ptr, 2, _lib.stream())
            _lib.call("cfm_probe_slot", ptr, 3, _lib.stream())

    def reset(self):
        self.slots.zero_()
        self.cal.zero_()

    def empty_pair_ms(self):
        n = int(self.cal[:, 3].sum().item())
        return (self.cal[:, 5].double().sum().item() / self.khz / n) if n else None

    def mean_ms(self, incl=False):
        """(mean ms per timed launch, launches timed): busy, or with incl=True the stamp-to-stamp interval minus
        the empty pairs' (uncorrected when no calibration ran, e.g. eager runs)."""
        torch.cuda.synchronize()
        tot = self.slots[:, 5 if incl else 2].double().sum().item()
        n = int(self.slots[:, 3].sum().item())
        if not n:
            return float("nan"), 0
        ms = tot / self.khz / n
        if incl and self.empty_pair_ms() is not None:
            ms -= self.empty_pair_ms()
        return ms, n

    def _mean(self, per_slot):
        cnt = self.slots[:, 3].double().cpu()
        n = cnt.sum().item()
        return (sum(f * c for f, c in zip(per_slot, cnt.tolist())) / n) if n else float("nan")

    def mean_flops(self):
        """Launch-weighted mean FLOPs per timed launch (a family of GEMM shapes)."""
        return self._mean(self.slot_flops)

    def mean_bytes(self):
        """Launch-weighted mean algorithmic bytes per timed launch (gemm_desc_bytes)."""
        return self._mean(self.slot_bytes)


def lib_md5():
    import hashlib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def trace_family_ms(summary_file, config, family):
    """The rocprofv3 kernel-trace figure of a kernel family, read from a committed summary
    (profiles/summarize_trace.py output: per (kernel, grid) rows of launches per step and mean duration) of a
    bench.py run of the same config: (mean ms per launch, launches per step, summary path, same build) or None;
    `same build`: the summary's libcfm.so md5 is the md5 of the library this run loaded."""
    path = os.path.join(REPO, summary_file)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        rec = json.load(f)
    if rec.get("config") != config:
        return None
    fam = rec.get("families", {}).get(family)
    if not fam:
        return None
    return fam["avg_ns"] / 1e6, fam["launches_per_step"], summary_file, rec.get("lib_md5") == lib_md5()


def time_ctc_head(h, reps=20):
    """The fused CTC head (Linear d->V + log_softmax + CTC loss, fwd + bwd, ctc.hip) alone at the step's shape,
    as one captured HIP graph replayed `reps` times (HIP events): its share of the timed step, which SURVEY.md
    §8d reports separately from the encoder metric.  Runs after the timed region on copies of the head's
    weights (the model's gradients are untouched)."""
    m = h.model
    M = h.B * h.T2
    g = torch.Generator(device="cpu").manual_seed(7)
    y = (torch.randn(M, h.d, generator=g) * 0.5).to(h.dev).requires_grad_()
    w = m.ctc_fc.weight.detach().clone().requires_grad_()
    b = m.ctc_fc.bias.detach().clone().requires_grad_()

    def run():
        loss, _ = ctc_head_loss(y, w, b, h.tgt_i32, h.lens_i32, h.tlen_i32, h.B, h.T2, blank=0, reduction="mean",
                                zero_infinity=True, compute_dtype=m.cd)
        loss.backward()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            run()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    y.grad = w.grad = b.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        run()
    graph.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        graph.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def cgroup_cpu_quota():
    """CPUs this job may use per the cgroup v2 quota (cpu.max), or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def physical_cores():
    """(physical cores of the host, CPUs this process may run on): unique (physical id, core id) pairs of
    /proc/cpuinfo, and the scheduler affinity mask."""
    cores, phys, core = set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                elif not line.strip() and core is not None:
                    cores.add((phys, core))
                    phys = core = None
        if core is not None:
            cores.add((phys, core))
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return len(cores) or (os.cpu_count() or 1), aff


def cpu_model():
    """The host CPU's model name (reported next to the CPU baseline)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, threads, steps=3):
    """The CPU oracle (torch fp32 restatement of the same composition) on a bounded sample:
    1 utterance of the config's length through front-end + encoder + CTC, fwd+bwd, 1 warm-up then
    the best of `steps` timed steps."""
    from oracle import conformer as oc
    from oracle import frontend as of
    name, L, d, H, ffn, K, _, secs, pos = cfg
    torch.set_num_threads(threads)
    T_in = 100 * secs + 1
    g = torch.Generator().manual_seed(0)
    x = torch.rand(1, 1, 80, T_in, generator=g)
    w1 = (torch.randn(512, 1, 7, 7, generator=g) * 0.1).requires_grad_()
    b1 = torch.zeros(512, requires_grad=True)
    w2 = (torch.randn(128, 512, 3, 3, generator=g) * 0.01).requires_grad_()
    b2 = torch.zeros(128, requires_grad=True)
    T2 = ((T_in - 7) // 2 + 1 - 3) // 2 + 1
    wf = (torch.randn(d, 18 * 128, generator=g) * 0.02).requires_grad_()
    bf = torch.zeros(d, requires_grad=True)
    conf = oc.ConformerRef(d, H, ffn, L, K, 0.0, pos_enc=pos).train()
    wc = (torch.randn(1024, d, generator=g) * 0.02).requires_grad_()
    tgt = torch.randint(1, 1024, (1, T2 // 4), generator=g)
    lens = torch.tensor([T2])

    def step():
        h = of.frame_projection(of.convsub_forward(x, w1, b1, w2, b2), wf, bf)
        y, _ = conf(h, lens)
        lp = F.log_softmax(F.linear(y, wc), -1).transpose(0, 1)
        loss = F.ctc_loss(lp, tgt, lens, torch.tensor([T2 // 4]), blank=0, zero_infinity=True)
        loss.backward()

    step()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    dt = min(ts)
    return {"value": round(T_in / dt, 1), "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"{name} fp32 oracle (torch CPU), 1 x {secs} s utterance ({T_in} frames), front-end + "
                      f"{L} layers ({pos} pos) + CTC, fwd+bwd, best of {steps} steps after 1 warm-up"}


def cpu_baseline_s10(threads, steps=3):
    """BASELINE.json configs[0]: Conformer-S (16 L, d 144, 4 heads, ffn 576, K 31) forward on 4 x 10 s
    80-bin mel clips, the CPU plumbing path -- the fp32 oracle (front-end + frame projection + encoder),
    eval mode, no autograd."""
    from oracle import conformer as oc
    from oracle import frontend as of
    torch.set_num_threads(threads)
    B, T_in, d = 4, 1001, 144
    g = torch.Generator().manual_seed(1)
    x = torch.rand(B, 1, 80, T_in, generator=g)
    w1 = torch.randn(512, 1, 7, 7, generator=g) * 0.1
    b1 = torch.zeros(512)
    w2 = torch.randn(128, 512, 3, 3, generator=g) * 0.01
    b2 = torch.zeros(128)
    T2 = ((T_in - 7) // 2 + 1 - 3) // 2 + 1
    wf = torch.randn(d, 18 * 128, generator=g) * 0.02
    bf = torch.zeros(d)
    conf = oc.ConformerRef(d, 4, 576, 16, 31, 0.1).eval()
    lens = torch.full((B,), T2)
    with torch.no_grad():
        def fwd():
            return conf(of.frame_projection(of.convsub_forward(x, w1, b1, w2, b2), wf, bf), lens)
        fwd()
        ts = []
        for _ in range(steps):
            t0 = time.perf_counter()
            fwd()
            ts.append(time.perf_counter() - t0)
        dt = min(ts)
    return {"value": round(B * T_in / dt, 1), "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(),
            "sample": f"configs[0]: Conformer-S fp32 oracle forward (eval), 4 x 10 s clips ({T_in} frames), "
                      f"front-end + frame projection + 16 layers, best of {steps} after 1 warm-up"}


class Harness:
    """One training configuration of the bench, reusable by tests (tests/test_gpu_bench_harness.py) and the
    NaN hunt (benchmarks/nan_hunt.py): model + synthetic batch + GradAllReducer + Adafactor, the step as
    fwd_bwd() (captured into a HIP graph unless eager) + post() (all-reduce + optimizer, eager).

    Every step also adds (loss is not finite) to a device counter (`bad`, read once at the end, no host
    sync per step): the bench reports it as `nonfinite_steps` and exits non-zero when it is not 0."""

    def __init__(self, cfg, dev, rank=0, world=1, *, dropout=0.1, fp8=False, specaug=False, dp_overlap=False,
                 chunk_layers=4,
                 eager=False, no_optimizer=False, probe_inline=False, lr=2e-5, seed=1234, grad_bf16=False):
        self.cfg = cfg
        name, L, d, H, ffn, K, B, secs, pos_enc = cfg
        self.dev, self.rank, self.world = dev, rank, world
        self.eager = bool(eager)
        self.dp_overlap = bool(dp_overlap)
        self.no_optimizer, self.probe_inline = no_optimizer, probe_inline
        self.T_in, self.Fb, self.V = 100 * secs + 1, 80, 1024
        self.B, self.L, self.d, self.ffn = B, L, d, ffn
        self.cd = torch.bfloat16
        torch.manual_seed(seed)                      # identical init on every rank (then broadcast)
        self.model = EncoderCTC(L, d, H, ffn, K, self.V, self.Fb, self.T_in, dropout, self.cd, pos_enc,
                                fp8).to(dev).train()
        cdist.broadcast_parameters(self.model)
        self.params = [p for p in self.model.parameters() if p.requires_grad]
        # DP: the Conformer's grouped weight gradients are written straight into flat all-reduce buckets; with
        # dp_overlap each chunk's bucket is reduced while the lower layers' backward still runs (eager: from the
        # backward itself; graph: the step is captured as a chain of graphs cut at the chunk boundaries and the
        # reduces are issued between replays, cdist.SegmentedStepGraph).  grad_bf16: bf16 reduce copies
        self.reducer = cdist.GradAllReducer(self.params, model=self.model, overlap=bool(dp_overlap),
                                            grad_dtype=torch.bfloat16 if grad_bf16 else torch.float32,
                                            chunk_layers=chunk_layers)
        self.seg = None
        self.opt = Adafactor(self.params, lr=lr, beta1=0.9, scale_parameter=False, relative_step=False)
        # synthetic data: per-utterance min-max-normalised uniform mels, full lengths
        g = torch.Generator(device="cpu").manual_seed(seed + rank)
        x = torch.rand(B, self.Fb, self.T_in, generator=g)
        x = (x - x.amin((1, 2), keepdim=True)) / (x.amax((1, 2), keepdim=True) - x.amin((1, 2), keepdim=True))
        self.x = x.to(dev)
        self.T2 = T2 = self.model.T2
        self.lens_i32 = torch.full((B,), T2, dtype=torch.int32, device=dev)
        U = T2 // 4
        targets = torch.randint(1, self.V, (B, U), generator=g).to(dev)
        self.rng = torch.zeros(1, dtype=torch.int64, device=dev)     # device dropout step counter
        _lib.call("cfm_rng_bind", _lib.ptr(self.rng))
        self.tgt_i32 = targets.to(torch.int32).contiguous()
        self.tlen_i32 = torch.full((B,), U, dtype=torch.int32, device=dev)
        self.seed0 = 17 * rank + 1
        self.bad = torch.zeros(1, dtype=torch.int32, device=dev)     # steps whose loss was not finite
        self.one = torch.ones((), device=dev)                          # the loss gradient (no fill per step)
        set_nonfinite_counter(self.bad)     # the CTC mean's own launch counts non-finite losses (cfm_ctc_mean)
        self.ctc_aborts = torch.zeros(1, dtype=torch.int32, device=dev)   # recursion waits given up (cfm.h)
        _lib.call("cfm_ctc_bind_abort_counter", _lib.ptr(self.ctc_aborts))
        self.steps_run = 0
        # SpecAugment (configs[2]): the global batch's draws on the host in the reference's order
        # (specaugment.draw, python random seeded as speechcommands.py:18), this rank's slice packed into
        # a STATIC device block that the captured step reads; refreshed before every step
        self.sa_params = None
        if specaug:
            import random as _random
            self._sa_rng = _random.Random(42)
            self._sa_hp = HParams(None)
            self._tau_glob = [self.T_in] * (B * world)
            self.sa_params = self.specaug_refresh()
        self.graph = self.probe_graph = None
        self.static_loss = None
        self.host_t = []

    def specaug_refresh(self):
        B = self.B
        dr = specaugment.draw(B * self.world, self.Fb, self._tau_glob, self._sa_hp, self._sa_rng)
        blk = specaugment.pack(dr, self._tau_glob, self.rank * B, (self.rank + 1) * B)
        if self.sa_params is None:
            return blk.to(self.dev)
        self.sa_params.copy_(blk.pin_memory(), non_blocking=True)
        return self.sa_params

    def fwd_bwd(self):
        self.rng.add_(1)
        loss, _ = self.model(self.x, self.lens_i32, self.tgt_i32, self.tlen_i32, seed=self.seed0,
                             specaug_params=self.sa_params)
        loss.backward(self.one)
        return loss

    def post(self):
        self.reducer.allreduce()
        if not self.no_optimizer:
            self.opt.step()

    def setup(self, warmup, probes=()):
        """Eager: `warmup` steps.  Graph: warm up on a side stream (allocator + autotuned state settle), then
        capture ONE training step's forward + backward into a HIP graph (all-reduce + optimizer stay eager:
        few launches).  probes: KernelProbe objects -- a second capture of the same step carries their slot
        kernels and is replayed only after the timed region (probe_replays)."""
        opt = self.opt
        if self.eager:
            for _ in range(warmup):
                self.step()
            torch.cuda.synchronize()
            return
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 1)):
                opt.zero_grad(set_to_none=True)
                self.fwd_bwd()
                self.post()
                self.steps_run += 1
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        opt.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        if self.probe_inline:                 # legacy: probes inside the timed graph
            for p in probes:
                p.active = True
        if self.dp_overlap:
            self.seg = cdist.SegmentedStepGraph(self.reducer)
            self.static_loss = self.seg.capture(self.fwd_bwd)
        else:
            with torch.cuda.graph(self.graph):
                self.static_loss = self.fwd_bwd()
            self.reducer.mark_graph()
        for p in probes:
            p.active = False
        grads_timed = [p.grad for p in self.params]
        if probes and not self.probe_inline:
            # a second capture of the same step carries the probe's slot kernels (68 one-lane launches per
            # step); it is replayed after the timed region, so the probes never sit inside `value`'s clock
            opt.zero_grad(set_to_none=True)
            self.probe_graph = torch.cuda.CUDAGraph()
            for p in probes:
                p.active = True
            with self.reducer.no_sync(), torch.cuda.graph(self.probe_graph):    # (no reduce / cut inside)
                for p in probes:
                    p.calibrate()
                self.fwd_bwd()
            for p in probes:
                p.active = False
            for p, g in zip(self.params, grads_timed):
                p.grad = g           # the timed replays' optimizer steps read the timed graph's grads
        self.step()                  # one replay outside the timed region
        torch.cuda.synchronize()

    def step(self):
        if self.graph is None:
            self.opt.zero_grad(set_to_none=True)
            if self.sa_params is not None:
                self.specaug_refresh()
            loss = self.fwd_bwd()
            self.post()
            self.static_loss = loss
        else:
            t_a = time.perf_counter()
            if self.sa_params is not None:
                self.specaug_refresh()
            if self.seg is not None:
                self.seg.replay()
            else:
                self.graph.replay()
            t_b = time.perf_counter()
            self.post()
            self.host_t.append((t_b - t_a, time.perf_counter() - t_b))
        self.steps_run += 1
        return self.static_loss

    def probe_replays(self, n):
        if self.probe_graph is not None:
            for _ in range(n):
                self.probe_graph.replay()

    def nonfinite_steps(self):
        return int(self.bad.item())

    def close(self):
        """Unbind the device dropout counter (libcfm keeps its address; it dies with this harness)."""
        torch.cuda.synchronize()
        _lib.call("cfm_rng_bind", None)
        _lib.call("cfm_ctc_bind_abort_counter", None)
        set_nonfinite_counter(None)

    def params_finite(self):
        """All parameters finite (one pass over the weights; after the timed region)."""
        ok = torch.ones(1, dtype=torch.bool, device=self.dev)
        for p in self.params:
            ok &= torch.isfinite(p.detach()).all()
        return bool(ok.item())


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` run WITHOUT a torchrun environment: start N ranks of this same command under
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) as a CHILD process and exit with its code.
    The parent never touches the GPU (nothing before this point loads libcfm or calls HIP), so no process that
    initialised the device is replaced.  stdout lines that are JSON objects (rank 0's one result line) pass through
    to stdout; everything else the launcher prints goes to stderr."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    print("bench: launching", n, "ranks:", " ".join(cmd), file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        s = line.strip()
        is_json = s.startswith("{") and s.endswith("}")
        print(s if is_json else line.rstrip("\n"), file=sys.stdout if is_json else sys.stderr, flush=True)
    return proc.wait()


def check_launch(args, rank, world):
    """--check-launch: the process-group plumbing alone (no model, no kernels): every rank contributes 1 to one
    all-reduce; rank 0 prints the world the launcher built and the count the collective saw."""
    import torch.distributed as tdist
    backend = tdist.get_backend() if tdist.is_initialized() else None
    seen = 1
    if world > 1:
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        t = torch.ones(1, device=dev)
        tdist.all_reduce(t)
        seen = int(t.item())
    if rank == 0:
        print(json.dumps({"check": "launch", "n_gpus": world, "gpus_requested": args.gpus, "dist_backend": backend,
                          "world_size_reported": tdist.get_world_size() if tdist.is_initialized() else 1,
                          "ranks_in_allreduce": seen}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); N > 1 without a torchrun env spawns torch.distributed.run itself")
    ap.add_argument("--check-launch", action="store_true",
                    help="only build the process group and run one all-reduce (launcher test; no GPU work)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="L15", choices=sorted(CONFIGS))
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-optimizer", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: the host's physical cores, SURVEY.md §8d; a 16-thread "
                         "figure -- one GPU's CPU share on the pool -- is reported beside it)")
    ap.add_argument("--gemm-mode", type=int, default=int(os.environ["CFM_GEMM_MODE"]) if "CFM_GEMM_MODE" in os.environ
                    else None, help="cfm_gemm_set_mode value (A/B tuning; env CFM_GEMM_MODE)")
    ap.add_argument("--attn-mode", type=int, default=int(os.environ.get("CFM_ATTN_MODE", "0")),
                    help="cfm_attn_set_mode value (A/B tuning; env CFM_ATTN_MODE)")
    ap.add_argument("--eager", action="store_true", help="launch every kernel from Python (no HIP graph)")
    ap.add_argument("--specaug", action="store_true",
                    help="SpecAugment inside the step (host draws in the reference order, one warp+mask kernel)")
    ap.add_argument("--pos-enc", choices=("none", "rel"), default=None, help="override the config's pos encoding")
    ap.add_argument("--layers", type=int, default=None, help="override the config's layer count (debug runs)")
    ap.add_argument("--nst", action="store_true", help="configs[3]: the NST pseudo-label pass (eval fwd + decode)")
    ap.add_argument("--fp8", action="store_true",
                    help="configs[4]: forward FFN / QKV / out-projection GEMMs on fp8 e4m3 MFMA (backward bf16)")
    ap.add_argument("--dp-overlap", action="store_true",
                    help="bucket all-reduces overlapped with the backward (default when N>1): graph mode captures "
                         "the step as a chain of graphs cut at the gradient-chunk boundaries; with --eager the "
                         "reduces are issued from the backward itself")
    ap.add_argument("--no-dp-overlap", action="store_true",
                    help="N>1: one graph for fwd+bwd, every bucket reduced after the replay")
    ap.add_argument("--grad-bf16", action="store_true",
                    help="N>1: reduce the gradient buckets through bf16 copies (half the xGMI bytes)")
    ap.add_argument("--dp-chunk-layers", type=int, default=4,
                    help="layers per gradient bucket chunk (overlap mode: one graph cut + grouped-wgrad flush each)")
    ap.add_argument("--probe-inline", action="store_true",
                    help="put the roofline probe kernels inside the timed graph (default: a separate probed graph)")
    ap.add_argument("--poison", action="store_true",
                    help="debug: NaN-fill every torch.empty (deterministic algorithms + fill_uninitialized_memory)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        print(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks", file=sys.stderr)
        sys.exit(2)
    if args.check_launch:
        rank, world, _ = cdist.init_from_env()
        return check_launch(args, rank, world)
    if args.poison:
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.utils.deterministic.fill_uninitialized_memory = True
    if args.gemm_mode is not None:
        _lib.call("cfm_gemm_set_mode", args.gemm_mode)
    if args.attn_mode:
        _lib.call("cfm_attn_set_mode", args.attn_mode)

    rank, world, local = cdist.init_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = CONFIGS[args.config]
    if args.pos_enc is not None:
        cfg = cfg[:8] + (args.pos_enc,)
    if args.layers is not None:
        cfg = cfg[:1] + (args.layers,) + cfg[2:]
    name, L, d, H, ffn, K, B, secs, pos_enc = cfg

    if args.nst:
        torch.manual_seed(1234)
        T_in, Fb = 100 * secs + 1, 80
        model = EncoderCTC(L, d, H, ffn, K, 1024, Fb, T_in, args.dropout, torch.bfloat16, pos_enc,
                           args.fp8).to(dev).train()
        cdist.broadcast_parameters(model)
        gx = torch.Generator(device="cpu").manual_seed(1234 + rank)
        xs = torch.rand(B, Fb, T_in, generator=gx)
        xs = (xs - xs.amin((1, 2), keepdim=True)) / (xs.amax((1, 2), keepdim=True) - xs.amin((1, 2), keepdim=True))
        return run_nst(args, model, xs.to(dev), torch.full((B,), model.T2, dtype=torch.int32, device=dev), dev, cfg,
                       rank, world)

    h = Harness(cfg, dev, rank, world, dropout=args.dropout, fp8=args.fp8, specaug=args.specaug,
                dp_overlap=args.dp_overlap or (world > 1 and not args.no_dp_overlap), eager=args.eager,
                chunk_layers=args.dp_chunk_layers,
                no_optimizer=args.no_optimizer, probe_inline=args.probe_inline, grad_bf16=args.grad_bf16)
    model, T2, T_in = h.model, h.T2, h.T_in

    # dominant kernel: the FFN up-projection GEMM (M=B*T2, N=ffn, K=d, bf16, SiLU epilogue)
    M_ffn = B * T2
    # (the FFN down-projection's data-gradient GEMM has the same (M, N, K): match the forward's
    # bias + SiLU epilogue on K-major operands, not the shape alone)
    probe = KernelProbe(lambda kind, shape, dsc: kind == "gemm" and shape == (M_ffn, ffn, d) and dsc.act == 1
                        and not dsc.act_grad and dsc.a_kmajor and dsc.b_kmajor and dsc.dtype_ab == _lib.BF16, dev)
    # --fp8: every fp8 (MX e4m3) forward GEMM -- FFN up / down, QKV, out-projection -- as one family against the fp8 peak
    fprobe = KernelProbe(lambda kind, shape, dsc: kind == "gemm" and dsc.dtype_ab == _lib.FP8, dev)
    # second probed family: the grouped weight-gradient launch (one per step)
    wprobe = KernelProbe(lambda kind, shape, dsc: kind == "wgroup", dev)
    # the dominant kernel family (round-3 kernel trace): every bf16 GEMM with a d-wide output over the step's
    # tokens -- FFN-down / out-projection / pointwise-conv-2 forward, every d-wide data gradient (FFN-up, QKV,
    # out-projection, pointwise convs) and the folded front-end GEMM (batch x T2 rows)
    dprobe = KernelProbe(lambda kind, shape, dsc: kind == "gemm" and shape[1] == d and shape[0] * dsc.batch == M_ffn
                         and dsc.dtype_ab == _lib.BF16 and dsc.split_k <= 1 and dsc.a_kmajor and dsc.b_kmajor, dev)
    ops.PROBE = lambda kind, shape, dsc, launch: probe(kind, shape, dsc, lambda: wprobe(
        kind, shape, dsc, lambda: dprobe(kind, shape, dsc, lambda: fprobe(kind, shape, dsc, launch))))
    h.setup(args.warmup, probes=(probe, wprobe, dprobe, fprobe))
    for pr in (probe, wprobe, dprobe, fprobe):
        pr.reset()
    bad_before = h.nonfinite_steps()

    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    if h.graph is None:
        probe.active = wprobe.active = dprobe.active = fprobe.active = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = h.step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    probe.active = wprobe.active = dprobe.active = fprobe.active = False
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = tt.item()
    ms_step = 1000.0 * elapsed / args.steps
    if h.graph is not None and os.environ.get("BENCH_HOST_TIMING"):
        print("host ms per step (replay, post):", [(round(1e3 * a, 2), round(1e3 * b, 2)) for a, b in h.host_t],
              file=sys.stderr)
    frames_total = B * T_in * world * args.steps
    value = frames_total / elapsed
    # numerics of the timed steps: non-finite losses over every step run (warm-up included) and the final weights
    loss_val = float(loss.item())
    nonfinite = h.nonfinite_steps()
    params_ok = h.params_finite()
    if world > 1:
        tt = torch.tensor([nonfinite, 0 if params_ok else 1], device=dev, dtype=torch.int64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.SUM)
        nonfinite, params_ok = int(tt[0].item()), int(tt[1].item()) == 0

    h.probe_replays(args.steps)
    ops.PROBE = None
    if os.environ.get("BENCH_PROBE_DUMP"):
        torch.save(probe.slots.cpu(), os.environ["BENCH_PROBE_DUMP"])
    where = ("over --steps replays of a second capture of the same step that carries the probe kernels, run right "
             "after the timed region (the timed graph carries no probes)" if h.probe_graph is not None else
             "in the timed region" + (" (graph replays)" if h.graph is not None else ""))
    timing = ("avg_launch_ms_live: s_memrealtime of a one-lane stamp kernel right before each matching launch to that of "
              "one right after it, minus the same interval of empty stamp pairs (empty_pair_ms) -- the time the "
              "launch adds to the serial stream (dispatch ramp + execution + end-of-kernel completion), as "
              "rocprofv3's kernel trace counts it; avg_launch_ms_busy: first-workgroup start to last-workgroup end; "
              + where)
    gemm_flops = 2.0 * M_ffn * ffn * d
    # algorithmic bytes of one FFN up-projection launch: A (M x d) + W (ffn x d) bf16 reads, bias fp32,
    # y and the saved pre-activation (M x ffn each, bf16) written
    gemm_bytes = 2.0 * (M_ffn * d + ffn * d) + 4.0 * ffn + 2.0 * 2.0 * M_ffn * ffn
    _, dg_n = dprobe.mean_ms(incl=True)
    wg_shapes = [(d, ffn), (ffn, d)] * 2 + [(3 * d, d), (d, d), (2 * d, d), (d, d)]   # (N, K) per layer
    wg_flops = 2.0 * M_ffn * L * sum(n * k for n, k in wg_shapes)
    wg_bytes = L * sum(2.0 * M_ffn * (n + k) + 4.0 * n * k + 4.0 * n for n, k in wg_shapes)
    _, fpf = algorithmic_flops_per_frame(L, d, H, ffn, K, T_in, T2, model.F2, rel=pos_enc == "rel", B=B)
    fg = ops.ffold_geometry(B, 80, T_in, 512, 128, d, 7, 2, 3, 2, torch.bfloat16, True)
    xpf = executed_flops_per_frame(L, d, H, ffn, K, T_in, T2, rel=pos_enc == "rel", B=B, Kp=fg.Kp, T2p=fg.T2p)
    step_tflops = xpf * B * T_in / (ms_step * 1e-3) / 1e12
    ref_tflops = fpf * B * T_in / (ms_step * 1e-3) / 1e12
    ctc_ms = time_ctc_head(h) if rank == 0 else float("nan")

    cfg_key = args.config + ("+fp8" if args.fp8 else "") + ("+specaug" if args.specaug else "") + (
        f"+pos_{args.pos_enc}" if args.pos_enc else "") + (f"+L{args.layers}" if args.layers else "")

    def roofline_entry(kernel, flops, nbytes, pr, pmc_file, family, peak_tflops=PEAK_BF16_TFLOPS):
        """bound from the kernel's arithmetic intensity against the machine balance (peak FLOP/s over peak
        HBM B/s); `achieved`/`peak`/`frac` in that bound's unit, both fractions reported.  Duration per launch, three
        ways: live probes (dispatch-inclusive and busy, KernelProbe) and the rocprofv3 kernel-trace mean of the same
        family from a committed profiles/r05 summary of a bench.py run of this config.  `frac` uses the trace's mean
        when that summary was taken with THIS libcfm.so build (md5), so it reproduces from profiles/; otherwise the
        live dispatch-inclusive mean."""
        ms_live, n_launch = pr.mean_ms(incl=True)
        ms_busy, _ = pr.mean_ms()
        tr = None
        for rnd in ("r06", "r05"):      # this round's committed trace summary of the config, else the last round's
            tr = trace_family_ms(f"profiles/{rnd}/trace_{cfg_key}.json", cfg_key, family)
            if tr is not None:
                break
        use_trace = tr is not None and tr[3]
        ms = tr[0] if use_trace else ms_live
        intensity = flops / nbytes
        balance = peak_tflops * 1e12 / (PEAK_HBM_GBS * 1e9)
        tflops = flops / (ms * 1e-3) / 1e12
        gbs = nbytes / (ms * 1e-3) / 1e9
        hbm = intensity < balance
        e = {"kernel": kernel, "bound": "hbm" if hbm else "mfma",
             "achieved": round(gbs if hbm else tflops, 1), "peak": PEAK_HBM_GBS if hbm else peak_tflops,
             "unit": "GB/s" if hbm else "TFLOP/s",
             "frac": round(gbs / PEAK_HBM_GBS if hbm else tflops / peak_tflops, 4), "traffic": None,
             "mfma_frac": round(tflops / peak_tflops, 4), "mfma_peak_tflops": peak_tflops,
             "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
             "intensity_flop_per_byte": round(intensity, 1), "machine_balance_flop_per_byte": round(balance, 1),
             "avg_launch_ms": round(ms, 4),
             "duration_basis": "rocprofv3 kernel trace of this build (avg_launch_ms_trace)" if use_trace else
                               "live dispatch-inclusive probe (avg_launch_ms_live)",
             "avg_launch_ms_live": round(ms_live, 4), "avg_launch_ms_busy": round(ms_busy, 4),
             "empty_pair_ms": None if pr.empty_pair_ms() is None else round(pr.empty_pair_ms(), 4),
             "launches_timed": n_launch,
             "timing": timing, "flops_per_launch": flops, "algorithmic_bytes": nbytes}
        if tr is not None:
            e["avg_launch_ms_trace"] = round(tr[0], 4)
            e["trace_launches_per_step"] = tr[1]
            e["trace_same_build"] = tr[3]
            e["live_over_trace"] = round(ms_live / tr[0], 4)
            e["trace_source"] = tr[2] + " (rocprofv3 --kernel-trace of a bench.py run of this config: the family's "\
                                        "mean dispatch duration over the timed graph replays)"
        for rnd in ("r06", "r05", "r04", "r03", "r02"):
            path = os.path.join(REPO, "profiles", rnd, pmc_file)
            if not os.path.exists(path):
                continue
            with open(path) as f:
                rec = json.load(f)
            if rec.get("shape_key") == [M_ffn, d, ffn, L] and rec.get("hbm_bytes_per_launch"):
                e["traffic"] = rec["hbm_bytes_per_launch"]
                e["traffic_source"] = f"profiles/{rnd}/{pmc_file} ({rec.get('kernel', '?')[:80]})"
                if rec.get("algorithmic_bytes_per_launch"):
                    e["traffic_over_algorithmic"] = round(rec["hbm_bytes_per_launch"] /
                                                          rec["algorithmic_bytes_per_launch"], 3)
                    e["pmc_algorithmic_bytes"] = rec["algorithmic_bytes_per_launch"]
                break
        return e

    valid = nonfinite == 0 and params_ok
    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "mel-frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp8-e4m3 fwd GEMMs + bf16" if args.fp8 else "bf16",
        "data": "synthetic (uniform min-max-normalised 80-bin mels, random init)",
        "config": {"workload": f"{name} encoder fwd+bwd + CTC head, {B} x {secs} s utterances per GPU",
                   "model": name, "layers": L, "d_model": d, "heads": H, "ffn": ffn, "conv_kernel": K,
                   "pos_enc": pos_enc, "specaug": bool(args.specaug),
                   "global_batch": B * world, "seq_len": T_in, "enc_frames": T2, "frontend": "frame",
                   "dropout": args.dropout, "optimizer": None if args.no_optimizer else "adafactor",
                   "parallelism": f"dp{world}",
                   "launch": "eager" if h.eager else (f"hip-graph chain ({len(h.seg)} segments, bucket all-reduce "
                                                      "between replays)" if h.seg is not None
                                                      else "hip-graph (fwd+bwd)"),
                   "grad_reduce_dtype": "bf16" if h.reducer.grad_dtype == torch.bfloat16 else "fp32",
                   **({"dp_chunk_layers": args.dp_chunk_layers} if h.seg is not None else {})},
        "per_gpu_value": round(value / world, 1),
        "dist_backend": torch.distributed.get_backend() if torch.distributed.is_initialized() else None,
        "world_size_reported": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
        # FLOPs the step executes (encoder + the folded front-end GEMMs; CTC head excluded), and the reference
        # composition's count (conv1 + conv2 + projection as the reference computes them) beside it
        "step_executed_tflops": round(step_tflops, 1),
        "step_mfma_frac": round(step_tflops / PEAK_BF16_TFLOPS, 4),
        "step_flops_basis": "executed: encoder (SURVEY.md 8d per-layer MACs) + folded front-end GEMMs; CTC head "
                            "excluded (rounds 1-4 records named this key step_algorithmic_tflops; since round 4 it "
                            "is the executed count, the reference composition's is step_ref_composition_tflops)",
        "step_ref_composition_tflops": round(ref_tflops, 1),
        "ctc_head": {"ms": round(ctc_ms, 4), "share_of_step": round(ctc_ms / ms_step, 4),
                     "flops": 3 * 2.0 * B * T2 * d * h.V,
                     "timing": "fused Linear + log_softmax + CTC fwd+bwd alone at the step's shape, one HIP graph "
                               "replayed 20x after the timed region (HIP events); it runs inside the timed step"},
        "loss": loss_val,
        "steps_checked": h.steps_run, "nonfinite_steps": nonfinite, "nonfinite_before_timing": bad_before,
        "ctc_recursion_aborts": int(h.ctc_aborts.item()),
        "params_finite": params_ok, "valid": valid,
        # the dominant kernel family: d-wide-output GEMMs (mean FLOP / mean launch; bytes per launch from its
        # descriptor (gemm_desc_bytes): A + B read, C written in its dtype -- bf16 data gradients, fp32
        # residual-stream forwards written + residual read -- averaged likewise)
        "roofline": roofline_entry(f"gemm_ws (warp-specialised) d-wide outputs (N={d}, M={M_ffn} tokens): FFN-down / out-proj / pw2 "
                                   f"forward + every d-wide data gradient + the front-end fold, {dg_n // max(1, args.steps)}"
                                   f" launches per step", dprobe.mean_flops(), dprobe.mean_bytes(), dprobe,
                                   "gemm_dwide_pmc.json", "dwide"),
        "roofline_ffn_up": roofline_entry(f"gemm_pipe FFN up-projection M={M_ffn} N={ffn} K={d} (+bias+SiLU+dropout, "
                                          f"y and pre-activation stored)", gemm_flops, gemm_bytes, probe,
                                          "gemm_ffn_up_pmc.json", "ffn_up"),
        "roofline_wgrad": roofline_entry(f"grouped weight gradients (cfm_wgrad_group): {L} layers x 8 GEMMs, "
                                         f"M={M_ffn} tokens", wg_flops, wg_bytes, wprobe, "wgrad_group_pmc.json",
                                         "wgrad"),
    }
    if probe.mean_ms()[1] == 0:      # --fp8: the FFN up-projection runs on fp8 (roofline_fp8 below)
        del result["roofline_ffn_up"]
    if fprobe.mean_ms()[1] > 0:
        # the MX fp8 forward GEMM family (FFN up / down, QKV, out-projection; mean FLOP and descriptor bytes per
        # launch) against the ~5 PF dense fp8 peak
        result["roofline_fp8"] = roofline_entry(
            f"MX e4m3 forward GEMMs (v_mfma_scale_f32_32x32x64_f8f6f4, gemm_pipe F8): FFN up / down, QKV, out-projection, "
            f"{fprobe.mean_ms()[1] // max(1, args.steps)} launches per step", fprobe.mean_flops(), fprobe.mean_bytes(),
            fprobe, "gemm_fp8_pmc.json", "fp8", peak_tflops=PEAK_FP8_TFLOPS)
    if args.poison:
        result["poison"] = True
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # thread sweep up to the host's physical cores (64 per socket on the pool's EPYC 9575F); the job's CPU
        # quota (cgroup cpu.max) may be far below that, so the fastest count is the baseline and the sweep is
        # reported beside it
        phys, aff = physical_cores()
        quota = cgroup_cpu_quota()
        counts = [args.cpu_threads] if args.cpu_threads else sorted({t for t in (16, 32, 64) if t <= phys} or {phys})
        sweep = {t: cpu_baseline(cfg, t) for t in counts}
        best = max(sweep, key=lambda t: sweep[t]["value"])
        result["cpu_baseline"] = dict(sweep[best], host_physical_cores=phys, affinity_cpus=aff,
                                      cgroup_cpu_quota=quota,
                                      thread_sweep={str(t): v["value"] for t, v in sweep.items()})
        result["cpu_baseline_configs0"] = cpu_baseline_s10(best)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    if not valid:
        print(f"bench: INVALID step numerics: {nonfinite} of {h.steps_run} steps had a non-finite loss, "
              f"parameters finite: {params_ok}", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
