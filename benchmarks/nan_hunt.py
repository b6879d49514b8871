"""Find where a training step of the bench goes non-finite.

    python benchmarks/nan_hunt.py --config L15 [--layers N] [--eager] [--poison] [--steps 12]

Runs bench.Harness (the bench's own model / data / GradAllReducer / Adafactor / graph capture + probe capture)
and, after EVERY step, synchronises and reports: the loss, which parameter gradients are non-finite (before
the optimizer step), and whether every parameter is still finite after it.  --poison NaN-fills every
torch.empty (torch deterministic mode + fill_uninitialized_memory), so a kernel that reads memory nobody
wrote this step shows up deterministically.  With --eager and CFM_NANCHECK=1 the Conformer layers also name
their first non-finite intermediate (nn_conformer_for_speech_recognition_amd/debug.py)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from nn_conformer_for_speech_recognition_amd import debug  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="L15", choices=sorted(bench.CONFIGS))
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--probe", action="store_true", help="also capture the probe graph (as bench.py does)")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--no-optimizer", action="store_true")
    ap.add_argument("--disable", default="", help="CFM_DISABLE list for this run (set before import)")
    args = ap.parse_args()
    if args.poison:
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.utils.deterministic.fill_uninitialized_memory = True
    cfg = bench.CONFIGS[args.config]
    if args.layers is not None:
        cfg = cfg[:1] + (args.layers,) + cfg[2:]
    if args.batch is not None:
        cfg = cfg[:6] + (args.batch,) + cfg[7:]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    h = bench.Harness(cfg, dev, dropout=args.dropout, eager=args.eager, no_optimizer=args.no_optimizer)
    names = {id(p): n for n, p in h.model.named_parameters()}
    probes = ()
    if args.probe:
        M = h.B * h.T2
        pr = bench.KernelProbe(lambda kind, shape, dsc: kind == "gemm" and shape == (M, h.ffn, h.d), dev)
        wp = bench.KernelProbe(lambda kind, shape, dsc: kind == "wgroup", dev)
        bench.ops.PROBE = lambda kind, shape, dsc, launch: pr(kind, shape, dsc, lambda: wp(kind, shape, dsc, launch))
        probes = (pr, wp)
    report = {"config": cfg, "eager": args.eager, "poison": args.poison, "probe": args.probe, "steps": []}

    def snapshot():
        snap = {}
        for p in h.params:
            st = h.opt.state.get(p, {})
            snap[id(p)] = (p.detach().clone(), None if p.grad is None else p.grad.detach().clone(),
                           {k: v.clone() for k, v in st.items() if torch.is_tensor(v)}, int(st.get("step", 0)))
        return snap

    def diagnose(snap):
        """After a post() that left non-finite weights: which parameters, and what a plain torch Adafactor
        (transformers' formulas, fp32) computes from the same pre-step weights / gradients / state."""
        out = []
        for p in h.params:
            if bool(torch.isfinite(p.detach()).all()):
                continue
            p0, g0, st0, step0 = snap[id(p)]
            rec = {"name": names[id(p)], "shape": list(p.shape), "grad_finite": bool(torch.isfinite(g0).all()),
                   "p0_finite": bool(torch.isfinite(p0).all()), "state_finite": {k: bool(torch.isfinite(v).all())
                                                                                 for k, v in st0.items()},
                   "step_before": step0, "grad_ptr": p.grad.data_ptr(), "n_bad": int((~torch.isfinite(p)).sum())}
            try:
                from transformers.optimization import Adafactor as HFA
                q = torch.nn.Parameter(p0.clone())
                q.grad = g0.clone()
                o = HFA([q], lr=2e-5, beta1=0.9, scale_parameter=False, relative_step=False)
                if step0:
                    o.state[q] = {"step": step0, **{k: v.clone() for k, v in st0.items()}}
                    o.state[q]["RMS"] = 0
                o.step()
                rec["hf_finite"] = bool(torch.isfinite(q.detach()).all())
            except Exception as e:        # noqa: BLE001
                rec["hf_error"] = repr(e)[:200]
            out.append(rec)
            if len(out) >= 6:
                break
        return out

    def inspect(i, loss):
        torch.cuda.synchronize()
        lv = float(loss.item())
        bad_g = [names[id(p)] for p in h.params if p.grad is not None and not bool(torch.isfinite(p.grad).all())]
        none_g = [names[id(p)] for p in h.params if p.grad is None]
        return {"step": i, "loss": lv, "nonfinite_grads": bad_g[:12], "n_nonfinite_grads": len(bad_g),
                "missing_grads": none_g[:6]}

    # warm-up / capture exactly as bench.py (graph mode), then per-step inspection
    if h.eager:
        for i in range(args.warmup + args.steps):
            debug.reset()
            h.opt.zero_grad(set_to_none=True)
            loss = h.fwd_bwd()
            rec = inspect(i, loss)
            h.post()
            torch.cuda.synchronize()
            rec["params_finite_after"] = h.params_finite()
            rec["nancheck_first"] = debug.HITS[:8]
            report["steps"].append(rec)
            print(json.dumps(rec), flush=True)
    else:
        h.setup(args.warmup, probes=probes)
        rec = inspect(-1, h.static_loss)
        rec["params_finite_after"] = h.params_finite()
        print(json.dumps(rec), flush=True)
        for i in range(args.steps):
            h.graph.replay()
            rec = inspect(i, h.static_loss)
            snap = snapshot()
            rec["fast_path_key_hit"] = any(v[0] == h.opt._ptrkey([p for p in g["params"] if p.grad is not None])
                                           for g in h.opt.param_groups for v in [h.opt._fast.get((id(g), dev))]
                                           if v is not None)
            h.post()
            torch.cuda.synchronize()
            rec["params_finite_after"] = h.params_finite()
            if not rec["params_finite_after"]:
                rec["diagnose"] = diagnose(snap)
            report["steps"].append(rec)
            print(json.dumps(rec), flush=True)
            if args.probe and i % 3 == 2:
                h.probe_replays(1)       # interleave the probe graph (bench replays it after the timed loop)
    n_bad = sum(1 for r in report["steps"] if r["loss"] != r["loss"] or r["n_nonfinite_grads"])
    print(json.dumps({"summary": True, "config": cfg[0], "layers": cfg[1], "eager": args.eager,
                      "poison": args.poison, "bad_steps": n_bad, "total": len(report["steps"]),
                      "counter": h.nonfinite_steps()}), flush=True)
    sys.exit(1 if n_bad else 0)


if __name__ == "__main__":
    main()
