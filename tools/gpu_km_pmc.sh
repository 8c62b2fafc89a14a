# PMC passes over the KMeans kernel bench (one counter group per run; never combined with trace domains)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
for v in 7; do
  for mode in "" "--compute-only"; do
    tag=v${v}${mode:+_co}
    timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $R/gpurun_out/pmc/${tag}_p1 -o p1 -- python3 $R/tools/kmeans_kernel_bench.py --rows 100000000 --iters 2 $mode > $R/gpurun_out/pmc/${tag}_p1.log 2>&1 || { tail -5 $R/gpurun_out/pmc/${tag}_p1.log; exit 1; }
  done
  timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $R/gpurun_out/pmc/v${v}_p2 -o p2 -- python3 $R/tools/kmeans_kernel_bench.py --rows 100000000 --iters 2  > $R/gpurun_out/pmc/v${v}_p2.log 2>&1 || { tail -5 $R/gpurun_out/pmc/v${v}_p2.log; exit 1; }
done
echo PMC_OK
