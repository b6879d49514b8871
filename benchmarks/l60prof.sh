set -o pipefail
mkdir -p gpurun_out/l60
bash benchmarks/prof_bench.sh gpurun_out/l60/bf16.csv --config L60 --steps 4 --warmup 2 --no-cpu-baseline && \
python profiles/summarize.py gpurun_out/l60/bf16.csv auto 30 > gpurun_out/l60/bf16.txt && \
bash benchmarks/prof_bench.sh gpurun_out/l60/fp8.csv --config L60 --fp8 --steps 4 --warmup 2 --no-cpu-baseline && \
python profiles/summarize.py gpurun_out/l60/fp8.csv auto 40 > gpurun_out/l60/fp8.txt && cat gpurun_out/l60/bf16.txt gpurun_out/l60/fp8.txt
