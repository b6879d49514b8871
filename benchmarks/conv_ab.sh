#!/bin/bash
# same-box A/B of the conv-module kernels: libcfm_base.so (A) vs libcfm.so (B), interleaved
set -o pipefail
O=$(pwd)/gpurun_out/conv_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conformer.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit 1; }
for r in 1 2 3; do
  CFM_LIB=$(pwd)/nn_conformer_for_speech_recognition_amd/libcfm_base.so timeout -k 10 60 python3 benchmarks/conv_probe.py 50 | sed "s/^/A /" || exit 1
  timeout -k 10 60 python3 benchmarks/conv_probe.py 50 | sed "s/^/B /" || exit 1
done
bash benchmarks/prof_bench_cmd.sh $O/stats.csv python3 $(pwd)/benchmarks/conv_probe.py 20 && python3 profiles/summarize.py $O/stats.csv 21 4
