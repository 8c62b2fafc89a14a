# v7 diagnostics: which part of the compute costs what (compute-only and full), k=100
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${KM_VARIANTS:-base noarg noacc nodist}; do
  if [ $v = base ]; then unset ALINK_HIP_LIB; else export ALINK_HIP_LIB=$PWD/alink_amd/ops/exp/libalink_hip_$v.so; fi
  for m in "" "--compute-only"; do
    timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --k 100 --iters 7 $m > gpurun_out/kmd_$v.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/kmd_$v.log; exit 1; }
    echo "$v $m $(tail -1 gpurun_out/kmd_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["hip_ms"],3), "ms")')"
  done
done
