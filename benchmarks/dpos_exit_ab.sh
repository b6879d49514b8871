set -e
mkdir -p gpurun_out/r06q
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread -k "rel" > gpurun_out/r06q/tests3.log 2>&1
for r in 1 2 3; do
  for lib in ab/libcfm_base.so ""; do
    echo "[${lib:-new}] $(CFM_LIB=$lib timeout -k 10 120 python benchmarks/rel_modes.py --modes 0 --reps 3 | grep REL)"
  done
done > gpurun_out/r06q/dpos_ab.txt
cd /tmp && export TMPDIR=/tmp
for lib in /root/repo/ab/libcfm_base.so ""; do
  CFM_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/r06q/ab_${lib:+base} -o run -- python3 /root/repo/benchmarks/rel_modes.py --modes 0 --reps 2 > /dev/null 2>&1
done
