"""Potential of running the L15 step as two half-batch streams: one B=32 step graph vs two B=16 step graphs
replayed back to back on one stream vs the two replayed concurrently on two streams (forward + backward only, no
optimizer; the two halves are independent models here -- a timing probe, not a training step: BatchNorm
statistics would need a join between the halves).
    python benchmarks/stream_pair_probe.py [--reps 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def timed(fn, reps):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--config", default="L15")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS[a.config]
    half = cfg[:6] + (cfg[6] // 2,) + cfg[7:]
    full = bench.Harness(cfg, dev, no_optimizer=True)
    full.setup(2)
    ha = bench.Harness(half, dev, no_optimizer=True, seed=1)
    ha.setup(2)
    hb = bench.Harness(half, dev, no_optimizer=True, seed=2)
    hb.setup(2)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def pair_serial():
        ha.graph.replay()
        hb.graph.replay()

    def pair_concurrent():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ha.graph.replay()
        with torch.cuda.stream(s2):
            hb.graph.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    res = {}
    for rnd in range(2):
        res[f"full_B{cfg[6]}_ms_{rnd}"] = round(timed(full.graph.replay, a.reps), 3)
        res[f"half_pair_serial_ms_{rnd}"] = round(timed(pair_serial, a.reps), 3)
        res[f"half_pair_concurrent_ms_{rnd}"] = round(timed(pair_concurrent, a.reps), 3)
        res[f"half_single_ms_{rnd}"] = round(timed(ha.graph.replay, a.reps), 3)
    print("PAIR", json.dumps(res))


if __name__ == "__main__":
    main()
