# KMeans v7 prefetch-depth sweep (experimental libs under alink_amd/ops/exp): k=100, 1e8 x 128 bf16
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${KM_VARIANTS:-base a3 a5 a6}; do
  if [ $v = base ]; then unset ALINK_HIP_LIB; else export ALINK_HIP_LIB=$PWD/alink_amd/ops/exp/libalink_hip_$v.so; fi
  timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --k 100 --iters 7 > gpurun_out/km_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/km_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/km_$v.log)"
done
