// Tree-ensemble prediction (SURVEY P10 "batched predict kernels") on CDNA4 (gfx950 / MI355X).
//
// Reference: A/operator/common/tree/predictors/TreeModelMapper.java:89-152 (Predict / ProcessMissing),
// GbdtModelMapper.java:40-85 (sum of leaf values), RandomForestModelMapper.java (average of leaf distributions),
// LabelCounter.add (weightSum += w; dist[i] += leaf.dist[i] * w).
//
// Rows arrive as CODES, not raw values (built by tree_codes_kernel below, models/tree/model.py): for every continuous
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
#include <stdlib.h>

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

// Tree-split walk (the default when the LDS fits): the one-wave kernel above is latency-bound at 2 waves per CU —
// a 1000-feature code row block takes 64 KiB of LDS, so only two 64-row blocks fit a CU.  Here a 256-thread
// block shares ONE staged code block between 4 waves: wave w walks trees w, w+4, ... of a group of TP2_G trees for
// the same 64 rows (4x the waves per CU for the same LDS) and records each (tree, row)'s leaf — or -1 when the walk
// meets a missing value / unmapped category — in an LDS table; then wave 0 adds the group's leaves in tree order
// (weight 1: a[i] + dv[i] * 1 == a[i] + dv[i]) and redoes a -1 tree with the reference's weighted fan-out in
// place.  The sums therefore run in exactly the one-wave kernel's order: bit-identical results.
constexpr int TP2_G = 64;
constexpr int TP2_WAVES = 4;

template <typename CT, int NDR>
__global__ __launch_bounds__(64 * TP2_WAVES) void tree_predict2_kernel(
    const CT* __restrict__ codes, int64_t n, int stride, const int4* __restrict__ nodes,
    const double* __restrict__ dist, int nd, const double* __restrict__ wsum, const int* __restrict__ cat, int catw,
    const int* __restrict__ roots, int ntrees, double* __restrict__ acc, double* __restrict__ wacc,
    int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr uint32_t MISS = (uint32_t)(CT)~(CT)0;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t row0 = (int64_t)blockIdx.x * TP_ROWS;
    const int nrows = n - row0 < TP_ROWS ? (int)(n - row0) : TP_ROWS;
    {
        const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(codes) + row0 * stride);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        const int nvec = nrows * stride / 16;
        for (int e = tid; e < nvec; e += 64 * TP2_WAVES) dst[e] = src[e];
    }
    int* leafbuf = reinterpret_cast<int*>(lds + TP_ROWS * stride);
    __syncthreads();
    const bool live = lane < nrows;
    const CT* rc = reinterpret_cast<const CT*>(lds + lane * stride);
    const int64_t row = row0 + lane;
    double a[NDR > 0 ? NDR : 1];
    for (int i = 0; i < (NDR > 0 ? NDR : 1); ++i) a[i] = 0.0;
    double* ga = acc + row * nd;
    if (NDR == 0 && wave == 0 && live)
        for (int i = 0; i < nd; ++i) ga[i] = 0.0;
    double ws = 0.0;
    bool dead = false;
    for (int g0 = 0; g0 < ntrees; g0 += TP2_G) {
        const int gn = ntrees - g0 < TP2_G ? ntrees - g0 : TP2_G;
        if (live) {
            for (int j = wave; j < gn; j += TP2_WAVES) {
                int node = roots[g0 + j];
                int res;
                while (true) {
                    const int4 nv = nodes[node];
                    if (nv.x < 0) {
                        res = node;
                        break;
                    }
                    const uint32_t c = (uint32_t)rc[nv.x];
                    int child = -1;
                    if (c != MISS) {
                        if (nv.y >= 0) child = (int)c <= nv.y ? 0 : 1;
                        else if ((int)c < catw) child = cat[(int64_t)(-nv.y - 1) * catw + c];
                    }
                    if (child < 0) {
                        res = -1;
                        break;
                    }
                    node = nv.z + child;
                }
                leafbuf[j * TP_ROWS + lane] = res;
            }
        }
        __syncthreads();
        if (wave == 0 && live && !dead) {
            for (int j = 0; j < gn; ++j) {
                const int leaf = leafbuf[j * TP_ROWS + lane];
                if (leaf >= 0) {
                    ws += 1.0;
                    const double* dv = dist + (int64_t)leaf * nd;
                    if (NDR > 0) {
#pragma unroll
                        for (int i = 0; i < NDR; ++i) a[i] += dv[i];
                    } else {
                        for (int i = 0; i < nd; ++i) ga[i] += dv[i];
                    }
                    continue;
                }
                // the reference's weighted fan-out for this tree, depth first, added in place (one-wave kernel)
                int st_node[TP_STACK];
                double st_w[TP_STACK];
                int sp = 0, node = roots[g0 + j];
                double w = 1.0;
                while (true) {
                    const int4 nv = nodes[node];
                    if (nv.x < 0) {
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
                    double tot = 0.0;
                    for (int i = 0; i < nv.w; ++i) tot += wsum[nv.z + i];
                    if (tot == 0.0 || sp + nv.w - 1 > TP_STACK) {
                        atomicOr(err, tot == 0.0 ? 1 : 2);
                        dead = true;
                        break;
                    }
                    for (int i = nv.w - 1; i >= 1; --i) {
                        st_node[sp] = nv.z + i;
                        st_w[sp] = w * (wsum[nv.z + i] / tot);
                        ++sp;
                    }
                    w = w * (wsum[nv.z] / tot);
                    node = nv.z;
                }
                if (dead) break;
            }
        }
        __syncthreads();          // the leaf table is rewritten by the next group
    }
    if (wave == 0 && live && !dead) {
        if (NDR > 0)
#pragma unroll
            for (int i = 0; i < NDR; ++i) ga[i] = a[i];
        wacc[row] = ws;
    }
}

// ALINK_TREE_PREDICT_KERNEL=1 forces the one-wave kernel (A/B); default 2 = tree-split when its LDS fits
int tp_variant() {
    const char* e = getenv("ALINK_TREE_PREDICT_KERNEL");      // read per launch: tests A/B both in one process
    return (e != nullptr && e[0] == '1') ? 1 : 2;
}

template <typename CT>
int launch_tp(const void* codes, int64_t n, int stride, const void* nodes, const double* dist, int nd,
              const double* wsum, const int* cat, int catw, const int* roots, int ntrees, double* acc, double* wacc,
              int* err, hipStream_t st) {
    const int64_t blocks = (n + TP_ROWS - 1) / TP_ROWS;
    const CT* c = reinterpret_cast<const CT*>(codes);
    const int4* nv = reinterpret_cast<const int4*>(nodes);
    const size_t lds2 = (size_t)TP_ROWS * stride + (size_t)TP2_G * TP_ROWS * sizeof(int);
    if (lds2 <= 160 * 1024 && tp_variant() == 2) {
#define TP2_LAUNCH(NDR)                                                                                            \
    do {                                                                                                           \
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(tree_predict2_kernel<CT, NDR>),                    \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2) != hipSuccess)              \
            return 3;                                                                                              \
        hipLaunchKernelGGL((tree_predict2_kernel<CT, NDR>), dim3((unsigned)blocks), dim3(64 * TP2_WAVES), lds2,   \
                           st, c, n, stride, nv, dist, nd, wsum, cat, catw, roots, ntrees, acc, wacc, err);        \
    } while (0)
        switch (nd) {
            case 1: TP2_LAUNCH(1); break;
            case 2: TP2_LAUNCH(2); break;
            case 3: TP2_LAUNCH(3); break;
            case 4: TP2_LAUNCH(4); break;
            default: TP2_LAUNCH(0); break;
        }
#undef TP2_LAUNCH
        return hipGetLastError() == hipSuccess ? 0 : 2;
    }
    const size_t lds = (size_t)TP_ROWS * stride;
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

// Row codes for the walk above, on the device (replaces a batched searchsorted + scatter): block = TC_ROWS = 16 rows
// x 16 feature phases (256 threads).  A thread reads its column value (a wave covers 4 features x 16 consecutive
// rows: 128-byte segments), counts the feature's thresholds below it by a branchless binary search over a
// power-of-two row of the threshold table (+inf padded; W >= #thresholds + 1, so the count is exact:
// x <= thr_k <=> code <= k) and writes the code into an LDS tile of the rows' code vectors, which then goes out in
// 16-byte stores.  Two features per thread at a time (independent searches interleave), and only 16 rows of LDS
// per block (16 KiB at 1000 features) so ~8 blocks share a CU: the dependent threshold loads are latency-bound,
// occupancy is what hides them (round 6: a 64-row tile left 2 blocks per CU, 10.8 ms per 5e5 x 1000 rows).
// NaN -> MISS.  Slots the kernel does not own (categorical features) are left 0 for the caller to fill.
constexpr int TC_ROWS = 16;
constexpr int TC_PH = 256 / TC_ROWS;

template <typename CT>
__global__ __launch_bounds__(256) void tree_codes_kernel(const double* const* __restrict__ cols, int fc,
                                                         const int* __restrict__ slots,
                                                         const double* __restrict__ T, int W, int64_t row0,
                                                         int64_t n, int stride, CT* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr CT MISS = (CT)~(CT)0;
    const int tid = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * TC_ROWS;
    const int nrows = n - r0 < TC_ROWS ? (int)(n - r0) : TC_ROWS;
    const int nvec = TC_ROWS * stride / 16;
    uint4* tile = reinterpret_cast<uint4*>(lds);
    for (int e = tid; e < nvec; e += 256) tile[e] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const int r = tid % TC_ROWS;
    if (r < nrows) {
        CT* rc = reinterpret_cast<CT*>(lds + r * stride);
        const int64_t row = row0 + r0 + r;
        int f = tid / TC_ROWS;
        for (; f + TC_PH < fc; f += 2 * TC_PH) {
            const int g = f + TC_PH;
            const double x0 = cols[f][row], x1 = cols[g][row];
            const double* t0 = T + (int64_t)f * W;
            const double* t1 = T + (int64_t)g * W;
            int lo0 = 0, lo1 = 0;
            for (int s = W >> 1; s >= 1; s >>= 1) {
                const double a0 = t0[lo0 + s - 1], a1 = t1[lo1 + s - 1];
                lo0 += a0 < x0 ? s : 0;
                lo1 += a1 < x1 ? s : 0;
            }
            rc[slots[f]] = x0 != x0 ? MISS : (CT)lo0;
            rc[slots[g]] = x1 != x1 ? MISS : (CT)lo1;
        }
        if (f < fc) {
            const double x = cols[f][row];
            const double* t = T + (int64_t)f * W;
            int lo = 0;
            for (int s = W >> 1; s >= 1; s >>= 1) lo += t[lo + s - 1] < x ? s : 0;
            rc[slots[f]] = x != x ? MISS : (CT)lo;
        }
    }
    __syncthreads();
    uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<char*>(out) + r0 * stride);
    const int nv = nrows * stride / 16;
    for (int e = tid; e < nv; e += 256) dst[e] = tile[e];
}

}  // namespace

extern "C" {

// out [n][stride bytes] codes of rows row0 .. row0+n-1: for cont feature f (device pointer cols[f] to an fp64 column,
// NaN = NULL) the count of T[f][0..W) below the value at byte/short slot slots[f]; T rows are ascending, +inf padded,
// W a power of two > every feature's threshold count.  Other slots are zeroed.
int alink_tree_codes(const void* cols, int fc, const int* slots, const double* T, int W, int64_t row0, int64_t n,
                     int stride, int code_bytes, void* out, void* stream) {
    if (n <= 0) return 0;
    if (fc < 0 || W < 1 || (W & (W - 1)) != 0 || stride <= 0 || stride % 16 != 0 ||
        (int64_t)stride * TC_ROWS > 64 * 1024 || (code_bytes != 1 && code_bytes != 2))
        return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t lds = (size_t)TC_ROWS * stride;
    const unsigned blocks = (unsigned)((n + TC_ROWS - 1) / TC_ROWS);
    const double* const* c = reinterpret_cast<const double* const*>(cols);
    if (code_bytes == 1) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(tree_codes_kernel<uint8_t>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return 3;
        hipLaunchKernelGGL(tree_codes_kernel<uint8_t>, dim3(blocks), dim3(256), lds, st, c, fc, slots, T, W, row0, n,
                           stride, reinterpret_cast<uint8_t*>(out));
    } else {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(tree_codes_kernel<uint16_t>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return 3;
        hipLaunchKernelGGL(tree_codes_kernel<uint16_t>, dim3(blocks), dim3(256), lds, st, c, fc, slots, T, W, row0, n,
                           stride, reinterpret_cast<uint16_t*>(out));
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

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
