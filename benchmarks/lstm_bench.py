"""Time the libcfm BiLSTM decoder (csrc/lstm.hip) against torch.nn.LSTM (MIOpen) on the same GPU.

Shapes: the reference decoder nn.LSTM(256, 512, bidirectional=True) over one unbatched sequence of
L = B*T_enc steps (asrnn.py:38,252): L 1280 (native B 32 x 40 frames) and 11936 (L15: B 32 x 373).
Prints one JSON line per (impl, L) with forward and forward+backward ms."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
from nn_conformer_for_speech_recognition_amd.lstm import LSTM  # noqa: E402


def timeit(fn, n):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n


def main():
    dev = "cuda"
    only = sys.argv[1] if len(sys.argv) > 1 else None          # "libcfm": skip the MIOpen leg (profiling)
    for L in (1280, 11936):
        torch.manual_seed(0)
        ref = torch.nn.LSTM(256, 512, bidirectional=True).to(dev)
        mine = LSTM(256, 512, bidirectional=True).to(dev)
        mine.load_state_dict(ref.state_dict())
        x = torch.randn(L, 256, device=dev, requires_grad=True)
        dy = torch.randn(L, 1024, device=dev)
        n = 5 if L < 5000 else 2
        for name, m in (("libcfm", mine), ("torch_miopen", ref)):
            if only and name != only:
                continue
            def fwd():
                with torch.no_grad():
                    m(x)

            def fwdbwd():
                y, _ = m(x)
                y.backward(dy)
            f = timeit(fwd, n)
            fb = timeit(fwdbwd, n)
            print(json.dumps({"impl": name, "L": L, "fwd_ms": round(f, 3), "fwd_bwd_ms": round(fb, 3),
                              "us_per_step_fwd": round(f * 1e3 / L, 3)}), flush=True)


if __name__ == "__main__":
    main()
