#!/bin/bash
# same-box A/B of the conv-module kernels: libcfm_base.so (A) vs libcfm.so (B): parity tests on B, interleaved
# probe timings, and a rocprofv3 kernel summary of each
set -o pipefail
O=$(pwd)/gpurun_out/conv_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conformer.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit 1; }
A=$(pwd)/nn_conformer_for_speech_recognition_amd/libcfm_base.so
for r in 1 2 3; do
  CFM_LIB=$A timeout -k 10 60 python3 benchmarks/conv_probe.py 50 | sed "s/^/A /" || exit 1
  timeout -k 10 60 python3 benchmarks/conv_probe.py 50 | sed "s/^/B /" || exit 1
done
CFM_LIB=$A bash benchmarks/prof_bench_cmd.sh $O/statsA.csv python3 $(pwd)/benchmarks/conv_probe.py 20 && echo "A:" && python3 profiles/summarize.py $O/statsA.csv 21 3 && \
bash benchmarks/prof_bench_cmd.sh $O/statsB.csv python3 $(pwd)/benchmarks/conv_probe.py 20 && echo "B:" && python3 profiles/summarize.py $O/statsB.csv 21 3
