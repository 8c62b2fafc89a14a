# PMC counters of the KMeans kernel variants (k=100, 20M rows); summaries -> gpurun_out/prof_v5.txt
set -o pipefail
export TMPDIR=/tmp
P=/tmp/prof
mkdir -p $P gpurun_out
cd /tmp
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-5 4}; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d $P/a$v -o a$v -- python3 $R/tools/kmeans_kernel_bench.py --rows 20000000 --k 100 --iters 2 --variant $v > $P/a$v.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/b$v -o b$v -- python3 $R/tools/kmeans_kernel_bench.py --rows 20000000 --k 100 --iters 2 --variant $v > $P/b$v.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM --kernel-trace --output-format csv -d $P/c$v -o c$v -- python3 $R/tools/kmeans_kernel_bench.py --rows 20000000 --k 100 --iters 2 --variant $v > $P/c$v.log 2>&1 || echo "c$v failed"
done
python3 $R/tools/prof_summary.py $P $R/gpurun_out/prof_v5.txt > /dev/null
cat $R/gpurun_out/prof_v5.txt | grep -v reduce_slabs | head -120
