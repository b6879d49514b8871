#!/bin/bash
# LayerNorm backward A/B: base / two-row pipeline / residual-load hoist (interleaved), parity tests on each
set -o pipefail
P=$(pwd)/nn_conformer_for_speech_recognition_amd
for L in base ln2 lnh; do
  CFM_LIB=$P/libcfm_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layernorm or ln" 2>&1 | tail -1 | sed "s/^/$L tests: /"
done
for r in 1 2 3; do for L in base ln2 lnh; do CFM_LIB=$P/libcfm_$L.so timeout -k 10 60 python3 benchmarks/ln_probe.py 100 | sed "s/^/$L /" || exit 1; done; done
