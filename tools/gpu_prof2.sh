set -o pipefail
export TMPDIR=/tmp
P=/tmp/prof
mkdir -p $P gpurun_out
for k in 100 64; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d $P/a$k -o a$k -- python3 tools/kmeans_kernel_bench.py --rows 20000000 --k $k --iters 2 --variant 4 > $P/a$k.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/b$k -o b$k -- python3 tools/kmeans_kernel_bench.py --rows 20000000 --k $k --iters 2 --variant 4 > $P/b$k.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d $P/c$k -o c$k -- python3 tools/kmeans_kernel_bench.py --rows 20000000 --k $k --iters 2 --variant 4 > $P/c$k.log 2>&1 || echo "c$k failed"
done
python3 tools/prof_summary.py $P gpurun_out/prof_v4.txt > /dev/null
