set -e
cd /tmp && export TMPDIR=/tmp
O=${1:-/root/repo/gpurun_out/pmc_rel_dqs}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d /tmp/pa -o run -- python3 /root/repo/benchmarks/rel_modes.py --modes 0 --reps 1 > /dev/null 2>&1
cp $(find /tmp/pa -name '*counter_collection.csv' | head -1) $O/pa.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pb -o run -- python3 /root/repo/benchmarks/rel_modes.py --modes 0 --reps 1 > /dev/null 2>&1
cp $(find /tmp/pb -name '*counter_collection.csv' | head -1) $O/pb.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pc -o run -- python3 /root/repo/benchmarks/rel_modes.py --modes 0 --reps 1 > /dev/null 2>&1
cp $(find /tmp/pc -name '*counter_collection.csv' | head -1) $O/pc.csv
echo pmc done
