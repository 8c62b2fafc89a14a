// Fused score + running top-K of a query block against an item block — gfx950 / MI355X.
//
// Reference: BlockwiseCross.findTopK (A/operator/common/dataproc/BlockwiseCross.java:76-240) scores every
// (user, item) pair of a co-grouped block with a float sgemv and pushes it through a size-K PriorityQueue per
// user; AlsPredict.recommendForUsers (A/operator/common/recommendation/AlsPredict.java:32-103) is its only
// caller with a BLAS bulk score.  Here one launch merges a whole item block into the running top-K of every
// query, and the score matrix never exists in HBM:
//
//   * workgroup = 8 waves = 128 queries; wave w owns queries 16w..16w+15 of the block;
//   * item chunks of 64 rows are staged HBM -> registers -> LDS (prefetched one chunk ahead, row stride R+4
//     floats so the ds_read_b128 fragment reads are conflict-free) and shared by all 8 waves;
//   * scores on v_mfma_f32_16x16x4_f32 (exact f32: a fused-multiply-add chain, no bf16 rounding), A = 16
//     items x 4 dims, B = 4 dims x 16 queries; the query fragment stays in VGPRs for the whole launch.  The
//     k dimension is permuted (lane group g supplies dims 16s+4g+e) so one b128 read feeds 4 MFMAs;
//   * each query's top-K lives in LDS ([K][16] per wave, query-minor -> conflict-free scans) with its
//     current minimum as the admission threshold held in registers.  The common case is a wave-wide ballot
//     of "score > threshold" that comes back empty; candidates replace the minimum and trigger one
//     cooperative rescan (each lane group scans K/4 slots, two lane swaps combine them).
//
// The state (best_val / best_idx, [m][K], unsorted) is read at launch start and written at the end, so a
// ring of item blocks (parallel/cross.py) continues the same top-K across launches.  Ties keep the earlier
// entry (strict '>' admission, as the reference's PriorityQueue replace rule).
//
// Small query sets are split over items as well (grid.y = item slices, one state plane each, merged on the
// host by one topk over [m][slices*K]) so that a launch always has >= 2 workgroups per CU.
//
// Contract (checked by the host wrapper): R in {16, 32, 48, 64} (rank zero-padded), 1 <= K <= 128, Q [m][R]
// and T [n][R] row-major fp32, 16-B aligned; item indices (item_base + row) < 2^31.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int QW = 16;              // queries per wave
constexpr int WAVES = 8;
constexpr int QB = QW * WAVES;      // 128 queries per workgroup
constexpr int IT = 64;              // items per chunk
constexpr int KMAX = 128;

template <int R>
struct Cfg {
    static constexpr int STR = R + 4;                 // LDS row stride in floats
    static constexpr int TILE_F = IT * STR;
    static constexpr int LOADS = (IT * R / 4 + WAVES * 64 - 1) / (WAVES * 64);   // float4 loads / thread / chunk
};

// minimum (value, slot) of this lane's query over all K slots: lane group g scans slots g, g+4, ...
__device__ __forceinline__ void rescan(const float* tv, int K, int j, int g, float& thr, int& pos) {
    float mv = 3.4e38f;
    int mp = 0;
    for (int kk = g; kk < K; kk += 4) {
        const float v = tv[kk * QW + j];
        if (v < mv) { mv = v; mp = kk; }
    }
#pragma unroll
    for (int sh = 16; sh <= 32; sh <<= 1) {
        const float ov = __shfl_xor(mv, sh);
        const int op = __shfl_xor(mp, sh);
        if (ov < mv || (ov == mv && op < mp)) { mv = ov; mp = op; }
    }
    thr = mv;
    pos = mp;
}

// acc[b >> 2][b & 3] for a lane-varying b without dynamic register indexing (4 levels of selects)
__device__ __forceinline__ float pick16(const f32x4 (&acc)[4], int b) {
    const f32x4 lo = (b & 8) ? acc[2] : acc[0];
    const f32x4 hi = (b & 8) ? acc[3] : acc[1];
    const f32x4 v = (b & 4) ? hi : lo;
    const float a = (b & 2) ? v[2] : v[0];
    const float c = (b & 2) ? v[3] : v[1];
    return (b & 1) ? c : a;
}

template <int R>
__global__ __launch_bounds__(512) void topk_cross_kernel(const float* __restrict__ Q, int64_t m,
                                                         const float* __restrict__ T, int64_t n_all, int item_base,
                                                         int K, float* __restrict__ best_val,
                                                         int* __restrict__ best_idx, int64_t per_slice) {
    using C = Cfg<R>;
    // item slice blockIdx.y (split over items so small query sets still fill 256 CUs): its own state plane
    const int64_t i0 = (int64_t)blockIdx.y * per_slice;
    const int64_t n = n_all - i0 < per_slice ? n_all - i0 : per_slice;
    T += i0 * R;
    item_base += (int)i0;
    best_val += (int64_t)blockIdx.y * m * K;
    best_idx += (int64_t)blockIdx.y * m * K;
    __shared__ __attribute__((aligned(16))) float tile[C::TILE_F];
    __shared__ float topv[WAVES][KMAX * QW];
    __shared__ int topi[WAVES][KMAX * QW];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int j = lane & 15;
    const int g = lane >> 4;
    const int64_t q = (int64_t)blockIdx.x * QB + w * QW + j;
    const bool qok = q < m;
    float* tv = topv[w];
    int* ti = topi[w];

    // query fragment: lane (j, g) holds Q[q][16s + 4g + e]
    float qf[R / 4];
#pragma unroll
    for (int s = 0; s < R / 16; ++s) {
        f32x4 v = qok ? *reinterpret_cast<const f32x4*>(Q + q * R + 16 * s + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) qf[4 * s + e] = v[e];
    }
    // running state -> LDS (padding queries get +inf: nothing is ever admitted for them)
    for (int kk = g; kk < K; kk += 4) {
        tv[kk * QW + j] = qok ? best_val[q * K + kk] : 3.4e38f;
        ti[kk * QW + j] = qok ? best_idx[q * K + kk] : -1;
    }
    float thr;
    int pos;
    rescan(tv, K, j, g, thr, pos);

    const int64_t nchunks = (n + IT - 1) / IT;
    f32x4 pre[C::LOADS];
    auto load_chunk = [&](int64_t c) {
#pragma unroll
        for (int l = 0; l < C::LOADS; ++l) {
            const int e = (l * WAVES * 64 + tid) * 4;     // float offset inside the [IT][R] chunk
            const int64_t row = c * IT + e / R;
            pre[l] = (e < IT * R && row < n) ? *reinterpret_cast<const f32x4*>(T + row * R + (e % R))
                                             : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    if (nchunks > 0) load_chunk(0);
    for (int64_t c = 0; c < nchunks; ++c) {
        __syncthreads();                                  // previous chunk's reads are done
#pragma unroll
        for (int l = 0; l < C::LOADS; ++l) {
            const int e = (l * WAVES * 64 + tid) * 4;
            if (e < IT * R) *reinterpret_cast<f32x4*>(tile + (e / R) * C::STR + (e % R)) = pre[l];
        }
        __syncthreads();
        if (c + 1 < nchunks) load_chunk(c + 1);           // in flight while this chunk is scored

        f32x4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < R / 16; ++s) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(tile + (16 * t + j) * C::STR + 16 * s + 4 * g);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], qf[4 * s + e], acc[t], 0, 0, 0);
            }
        }
        // acc[t][r] = score(item 16t + 4g + r of the chunk, query j)
        const int64_t row0 = c * IT;
        uint32_t mask = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (acc[t][r] > thr && row0 + 16 * t + 4 * g + r < n) mask |= 1u << (4 * t + r);
        if (__ballot(mask != 0) == 0) continue;           // fast path: nothing beats any threshold
        // slow path: lane group by lane group (the 4 groups of a query must not race on its slots), each lane
        // walks only its own set bits
        for (int gg = 0; gg < 4; ++gg) {
            uint32_t mm = g == gg ? mask : 0u;
            while (__ballot(mm != 0u) != 0) {
                bool mine = false;
                float sc = 0.f;
                int idx = 0;
                if (mm != 0u) {
                    const int b = __builtin_ctz(mm);
                    mm &= mm - 1u;
                    sc = pick16(acc, b);
                    idx = item_base + (int)(row0 + 4 * g + 16 * (b >> 2) + (b & 3));
                    mine = sc > thr;
                }
                if (__ballot(mine) == 0) continue;
                if (mine) {
                    tv[pos * QW + j] = sc;
                    ti[pos * QW + j] = idx;
                }
                rescan(tv, K, j, g, thr, pos);
            }
        }
    }
    for (int kk = g; kk < K; kk += 4) {
        if (qok) {
            best_val[q * K + kk] = tv[kk * QW + j];
            best_idx[q * K + kk] = ti[kk * QW + j];
        }
    }
}

}  // namespace

extern "C" {

// Merge items T[0..n) (global ids item_base + row) into the running top-K of queries Q[0..m).
// best_val / best_idx: [slices][m][K] float / int32 states (init -inf / -1); item slice s (rows
// [s*per_slice, (s+1)*per_slice), per_slice a multiple of 64) is merged into plane s; unsorted on return.
int alink_topk_cross_f32(const float* Q, int64_t m, const float* T, int64_t n, int item_base, int R, int K,
                         float* best_val, int* best_idx, int slices, int64_t per_slice, void* stream) {
    if (m <= 0) return 0;
    if (K < 1 || K > KMAX || n < 0 || item_base < 0 || (int64_t)item_base + n > 0x7FFFFFFFLL) return -1;
    if (slices < 1 || per_slice % IT != 0 || (int64_t)(slices - 1) * per_slice >= (n > 0 ? n : 1)) return -3;
    const dim3 grid((unsigned)((m + QB - 1) / QB), (unsigned)slices);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (R) {
        case 16: hipLaunchKernelGGL(topk_cross_kernel<16>, grid, dim3(512), 0, st, Q, m, T, n, item_base, K, best_val, best_idx, per_slice); break;
        case 32: hipLaunchKernelGGL(topk_cross_kernel<32>, grid, dim3(512), 0, st, Q, m, T, n, item_base, K, best_val, best_idx, per_slice); break;
        case 48: hipLaunchKernelGGL(topk_cross_kernel<48>, grid, dim3(512), 0, st, Q, m, T, n, item_base, K, best_val, best_idx, per_slice); break;
        case 64: hipLaunchKernelGGL(topk_cross_kernel<64>, grid, dim3(512), 0, st, Q, m, T, n, item_base, K, best_val, best_idx, per_slice); break;
        default: return -2;
    }
    return (int)hipGetLastError();
}

}  // extern "C"
