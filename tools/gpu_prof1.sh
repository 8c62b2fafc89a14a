set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P=/tmp/prof
mkdir -p $P gpurun_out
cd /tmp && rocprofv3 -L > $P/counters_list.txt 2>&1; cd $R
grep -o "SQ_[A-Z_0-9]*\|TCC_[A-Z_0-9]*\|GRBM_[A-Z_0-9]*\|TCP_[A-Z_0-9]*" $P/counters_list.txt | sort -u > gpurun_out/counters_available.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/bench_trace -o bench -- python3 bench.py --steps 10 --warmup 2 --converge-iters 0 > $P/bench_trace.log 2>&1 && echo TRACE_OK
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $P/pmc1 -o pmc1 -- python3 tools/kmeans_kernel_bench.py --rows 20000000 --k 100 --iters 2 --variant 1 > $P/pmc1.log 2>&1 && echo PMC1_OK
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/pmc2 -o pmc2 -- python3 tools/kmeans_kernel_bench.py --rows 20000000 --k 100 --iters 2 --variant 1 > $P/pmc2.log 2>&1 && echo PMC2_OK
tail -3 $P/pmc2.log
python3 tools/prof_summary.py $P gpurun_out/prof_summary.txt > /dev/null
du -sh $P
