set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/diag.log
for s in 5 2 8; do timeout -k 10 200 python tools/kmeans_init_diag.py --iters 30 --init-steps $s >> gpurun_out/diag.log 2>&1 || exit 1; done
grep init_s gpurun_out/diag.log
timeout -k 10 200 python tools/kmeans_init_diag.py --rows 2000000 --iters 30 --init-steps 5 --torch 2>&1 | grep init_s
