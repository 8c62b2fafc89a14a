#!/bin/bash
# Build A/B variants of the v10 KMeans kernel into variants/libalink_hip_<name>.so (the in-tree lib's other
# objects + a variant kmeans_v10.o), for tools/kmeans_ab.py.  Run after `python build_native.py`.
#   pk       : one v_pk_add_f32 per row (accumulate body "pk")
#   pair     : -DKM10_PAIRMAX=1 (both distance tiles of a pair in one MFMA stage loop)
#   pkpair   : pk + pair
#   d16      : -DKM10_ACC_B32=0 (two ds_read_u16_d16_hi + two v_add_f32 per row; the default before round 4)
#   dot2     : -DKM10_ACC_B32=1 + body "dot2" (ds_read_b32 + 2 v_dot2_f32_bf16 per row; the default now)
#   dot2pair : dot2 + pair
#   timing   : -DKM10_TIMING=1 (per-workgroup wall-clock stamps; tools/kmeans_wg_timing.py).  `... timing` builds
#              only this one
#   pfd      : -DKM10_PFD=1 (the ALINK_KMEANS_V10_PFD L2 prefetch A/B; `... pfd` builds only this one)
set -e
cd "$(dirname "$0")/.."
mkdir -p variants
build_var() {
  name=$1; body=$2; flags=$3; d=build/variants/$name
  mkdir -p "$d"
  cp alink_amd/ops/csrc/kmeans_v10.hip alink_amd/ops/csrc/kmeans_tile.h "$d/"
  if [ "$body" = base ]; then cp alink_amd/ops/csrc/kmeans_v10_body.h "$d/"
  else python tools/gen_kmeans_v10_body.py --variant "$body" --out "$d/kmeans_v10_body.h"; fi
  (cd "$d" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 $flags \
      -c kmeans_v10.hip -o kmeans_v10.o)
  objs=$(ls build/hip/*.o | grep -v kmeans_v10)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "variants/libalink_hip_$name.so" $objs "$d/kmeans_v10.o"
}
[ "$1" = timing ] && { build_var timing base "-DKM10_TIMING=1"; exit 0; }
[ "$1" = pfd ] && { build_var pfd base "-DKM10_PFD=1"; exit 0; }
build_var d16 base "-DKM10_ACC_B32=0"
build_var pk pk "-DKM10_ACC_B32=0"
build_var pair base "-DKM10_ACC_B32=0 -DKM10_PAIRMAX=1"
build_var pkpair pk "-DKM10_ACC_B32=0 -DKM10_PAIRMAX=1"
build_var dot2 dot2 "-DKM10_ACC_B32=1"
build_var dot2pair dot2 "-DKM10_ACC_B32=1 -DKM10_PAIRMAX=1"
build_var timing base "-DKM10_TIMING=1"
build_var pfd base "-DKM10_PFD=1"
