// Tree-ensemble prediction (SURVEY P10 "batched predict kernels") on CDNA4 (gfx950 / MI355X).
//
// Reference: A/operator/common/tree/predictors/TreeModelMapper.java:89-152 (Predict / ProcessMissing),
// GbdtModelMapper.java:40-85 (sum of leaf values), RandomForestModelMapper.java (average of leaf distributions),
// LabelCounter.add (weightSum += w; dist[i] += leaf.dist[i] * w).
//
// Rows arrive as CODES, not raw values (built on the host side by models/tree/model.py): for every continuous
// feature the forest splits on, code = #{forest thresholds of that feature < x}, so "x <= threshold_k" is exactly
// "code <= k" (k = the threshold's rank); a categorical feature's code is its string-indexer index; MISS (the
// type's maximum) is a NULL / unseen value.  Codes are uint8 when every feature has < 255 thresholds / categories
// (the usual case: trained thresholds are bin boundaries), else uint16.
//
//   * one 64-lane workgroup per 64 rows; the rows' code vectors are staged in LDS once (16-byte copies) and every
//     tree is walked from LDS (the node table, 16 B per node, and leaf values stay in L2);
//   * a row's walk is the reference's recursion: a missing value (or a category mapped to no child) fans out over
//     all children with weight x child.weightSum / sum, depth first in child order, through a per-lane stack, so
//     leaf contributions are added in exactly the reference's order (trees in order, fp64 accumulate);
//   * node: {feature slot (-1 leaf), threshold rank k >= 0 or -(categorical map row)-1, first child, #children}.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int TP_ROWS = 64;
constexpr int TP_STACK = 48;

template <typename CT, int NDR>
__global__ __launch_bounds__(TP_ROWS) void tree_predict_kernel(const CT* __restrict__ codes, int64_t n, int stride,
                                                               const int4* __restrict__ nodes,
                                                               const double* __restrict__ dist, int nd,
                                                               const double* __restrict__ wsum,
                                                               const int* __restrict__ cat, int catw,
                                                               const int* __restrict__ roots, int ntrees,
                                                               double* __restrict__ acc, double* __restrict__ wacc,
                                                               int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr uint32_t MISS = (uint32_t)(CT)~(CT)0;
    const int tid = threadIdx.x;
    const int64_t row0 = (int64_t)blockIdx.x * TP_ROWS;
    const int nrows = n - row0 < TP_ROWS ? (int)(n - row0) : TP_ROWS;
    // stage this block's code rows (stride bytes each, a multiple of 16) into LDS
    {
        const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(codes) + row0 * stride);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        const int nvec = nrows * stride / 16;
        for (int e = tid; e < nvec; e += TP_ROWS) dst[e] = src[e];
    }
    __syncthreads();
    if (tid >= nrows) return;
    const CT* rc = reinterpret_cast<const CT*>(lds + tid * stride);
    const int64_t row = row0 + tid;
    double a[NDR > 0 ? NDR : 1];
    for (int i = 0; i < (NDR > 0 ? NDR : 1); ++i) a[i] = 0.0;
    double* ga = acc + row * nd;
    if (NDR == 0)
        for (int i = 0; i < nd; ++i) ga[i] = 0.0;
    double ws = 0.0;
    int st_node[TP_STACK];
    double st_w[TP_STACK];
    for (int t = 0; t < ntrees; ++t) {
        int sp = 0;
        int node = roots[t];
        double w = 1.0;
        while (true) {
            const int4 nv = nodes[node];
            if (nv.x < 0) {
                // leaf: LabelCounter.add(leaf.counter, w)
                ws += w;
                const double* dv = dist + (int64_t)node * nd;
                if (NDR > 0) {
#pragma unroll
                    for (int i = 0; i < NDR; ++i) a[i] += dv[i] * w;
                } else {
                    for (int i = 0; i < nd; ++i) ga[i] += dv[i] * w;
                }
                if (sp == 0) break;
                --sp;
                node = st_node[sp];
                w = st_w[sp];
                continue;
            }
            const uint32_t c = (uint32_t)rc[nv.x];
            int child = -1;
            if (c != MISS) {
                if (nv.y >= 0) child = (int)c <= nv.y ? 0 : 1;
                else if ((int)c < catw) child = cat[(int64_t)(-nv.y - 1) * catw + c];
            }
            if (child >= 0) {
                node = nv.z + child;
                continue;
            }
            // ProcessMissing: weights = child weightSum / their sum; child 0 now, the rest pushed in reverse
            double tot = 0.0;
            for (int i = 0; i < nv.w; ++i) tot += wsum[nv.z + i];
            if (tot == 0.0 || sp + nv.w - 1 > TP_STACK) {
                atomicOr(err, tot == 0.0 ? 1 : 2);
                return;
            }
            for (int i = nv.w - 1; i >= 1; --i) {
                st_node[sp] = nv.z + i;
                st_w[sp] = w * (wsum[nv.z + i] / tot);
                ++sp;
            }
            w = w * (wsum[nv.z] / tot);
            node = nv.z;
        }
    }
    if (NDR > 0)
#pragma unroll
        for (int i = 0; i < NDR; ++i) ga[i] = a[i];
    wacc[row] = ws;
}

template <typename CT>
int launch_tp(const void* codes, int64_t n, int stride, const void* nodes, const double* dist, int nd,
              const double* wsum, const int* cat, int catw, const int* roots, int ntrees, double* acc, double* wacc,
              int* err, hipStream_t st) {
    const int64_t blocks = (n + TP_ROWS - 1) / TP_ROWS;
    const size_t lds = (size_t)TP_ROWS * stride;
    const CT* c = reinterpret_cast<const CT*>(codes);
    const int4* nv = reinterpret_cast<const int4*>(nodes);
#define TP_LAUNCH(NDR)                                                                                             \
    do {                                                                                                           \
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(tree_predict_kernel<CT, NDR>),                     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)               \
            return 3;                                                                                              \
        hipLaunchKernelGGL((tree_predict_kernel<CT, NDR>), dim3((unsigned)blocks), dim3(TP_ROWS), lds, st, c, n,  \
                           stride, nv, dist, nd, wsum, cat, catw, roots, ntrees, acc, wacc, err);                  \
    } while (0)
    switch (nd) {
        case 1: TP_LAUNCH(1); break;
        case 2: TP_LAUNCH(2); break;
        case 3: TP_LAUNCH(3); break;
        case 4: TP_LAUNCH(4); break;
        default: TP_LAUNCH(0); break;
    }
#undef TP_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace

extern "C" {

// acc [n][nd] / wacc [n] (fp64) = the reference's LabelCounter of every row over the forest.  codes: [n] rows of
// `stride` bytes (multiple of 16, <= 160 KiB / 64), code_bytes 1 or 2.  *err |= 1 (a zero-weight fan-out: "Model is
// broken") or 2 (fan-out deeper than the per-lane stack; the caller falls back to the host walk).
int alink_tree_predict(const void* codes, int64_t n, int stride, int code_bytes, const void* nodes, const double* dist,
                       int nd, const double* wsum, const int* cat, int catw, const int* roots, int ntrees,
                       double* acc, double* wacc, int* err, void* stream) {
    if (n <= 0) return 0;
    if (stride <= 0 || stride % 16 != 0 || (int64_t)stride * TP_ROWS > 160 * 1024 || nd < 1 || ntrees < 0 ||
        (code_bytes != 1 && code_bytes != 2))
        return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    return code_bytes == 1
               ? launch_tp<uint8_t>(codes, n, stride, nodes, dist, nd, wsum, cat, catw, roots, ntrees, acc, wacc, err, st)
               : launch_tp<uint16_t>(codes, n, stride, nodes, dist, nd, wsum, cat, catw, roots, ntrees, acc, wacc, err,
                                     st);
}

}  // extern "C"
