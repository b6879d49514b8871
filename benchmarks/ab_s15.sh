set -o pipefail
B="python -u bench.py --config S15 --steps 20 --warmup 5 --no-cpu-baseline"
ms() { python -c "import json,sys; r=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$1', r['ms_per_step'])"; }
timeout -k 10 120 $B > gpurun_out/r06c/s15_def.json && ms gpurun_out/r06c/s15_def.json || exit 1
CFM_ATTN_MODE=64 timeout -k 10 120 $B > gpurun_out/r06c/s15_nosplit.json && ms gpurun_out/r06c/s15_nosplit.json || exit 1
CFM_GEMM_MODE=2097155 timeout -k 10 120 $B > gpurun_out/r06c/s15_pipe7.json && ms gpurun_out/r06c/s15_pipe7.json || exit 1
CFM_GEMM_MODE=524291 timeout -k 10 120 $B > gpurun_out/r06c/s15_nows.json && ms gpurun_out/r06c/s15_nows.json || exit 1
timeout -k 10 120 $B > gpurun_out/r06c/s15_def2.json && ms gpurun_out/r06c/s15_def2.json || exit 1
timeout -k 10 150 python -u bench.py --config M15 --specaug --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06c/m15.json && ms gpurun_out/r06c/m15.json || exit 1
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06c/l15.json && ms gpurun_out/r06c/l15.json
