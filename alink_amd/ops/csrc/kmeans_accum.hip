// KMeans per-cluster accumulation by a precomputed assignment (gfx950 / MI355X) — the general path.
//
// The fused v7 kernel (kmeans_v7.hip) covers the headline shape (bf16, D = 128, k <= 128, unweighted).  Every
// other bf16 shape — D in {64, 256} (D == 64 or a multiple of 128 up to 1024), k up to 256 (512 at D = 64),
// weighted rows
// (the reference's weighted KMeansAssignCluster, KMeansUtil.updateSumMatrix A/operator/common/clustering/kmeans/
// KMeansUtil.java:60-85) — runs as two passes: the MFMA nearest-centroid kernel (kmeans_nearest.hip) writes
// idx[N], then this kernel forms Sum[c][:] += w_r x_r and Cnt[c] += w_r.
//
// Layout: grid (row chunk b, dim slice s), DS = 128 dims per slice (64 when D == 64); a 512-thread workgroup
// keeps its slice of the k x DS fp32 partial sums in LDS (k <= 256 at DS = 128 -> 128 KiB, k <= 512 at DS = 64),
// 8 waves walk the chunk's rows, each lane loading DS/64 bf16 of a row (one coalesced 128/256-B wave load) and
// adding them with ds_add_f32 into row idx[r] of the LDS table (consecutive lanes -> consecutive banks, no
// conflicts; different rows of one wave never collide because a wave handles one row per instruction).
// Rows are prefetched 4 deep per wave (loads issued before the LDS adds of the previous group).  At the end
// the table goes to slab[b][c][D] (fp32) and a fixed-order fp64 reduction over chunks (kmeans_accum_reduce)
// forms [k][D+1].  Counts of unweighted rows are exact (integers < 2^24 per chunk); the fp32 sums inside a chunk
// depend on the LDS atomic order (rounding-level run-to-run differences, unlike v7's MFMA path).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int THREADS = 512;
constexpr int NW = THREADS / 64;
constexpr int PF = 4;                 // rows in flight per wave

template <int DS>
__global__ __launch_bounds__(THREADS) void kmeans_accum_kernel(const __bf16* __restrict__ X, int64_t N, int D,
                                                               const int* __restrict__ idx,
                                                               const float* __restrict__ w, int k,
                                                               int64_t rows_per_chunk, float* __restrict__ slab,
                                                               float* __restrict__ slab_cnt) {
    extern __shared__ float tab[];          // [k][DS] then cnt[k]
    constexpr int PER = DS / 64;            // dims per lane (1 or 2)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x, s = blockIdx.y;
    const int d0 = s * DS;
    float* cnt = tab + k * DS;
    for (int e = threadIdx.x; e < k * DS + k; e += THREADS) tab[e] = 0.f;
    __syncthreads();
    const int64_t r_lo = (int64_t)b * rows_per_chunk;
    const int64_t r_hi = r_lo + rows_per_chunk < N ? r_lo + rows_per_chunk : N;
    const bool do_cnt = s == 0 && lane == 0;
    for (int64_t r0 = r_lo + (int64_t)wave * PF; r0 < r_hi; r0 += (int64_t)NW * PF) {
        float xv[PF][PER];
        int c[PF];
        float wr[PF];
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int64_t r = r0 + q;
            const bool ok = r < r_hi;
            c[q] = ok ? idx[r] : -1;
            wr[q] = ok ? (w != nullptr ? w[r] : 1.f) : 0.f;
            const __bf16* xr = X + (ok ? r : r_lo) * D + d0 + PER * lane;
            if constexpr (PER == 2) {
                const uint32_t v = *reinterpret_cast<const uint32_t*>(xr);
                xv[q][0] = __uint_as_float(v << 16);
                xv[q][1] = __uint_as_float(v & 0xFFFF0000u);
            } else {
                xv[q][0] = (float)xr[0];
            }
        }
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int cq = __builtin_amdgcn_readfirstlane(c[q]);
            if (cq < 0 || cq >= k) continue;
            float* row = tab + cq * DS + PER * lane;
#pragma unroll
            for (int j = 0; j < PER; ++j)
                __hip_atomic_fetch_add(row + j, wr[q] * xv[q][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (do_cnt) __hip_atomic_fetch_add(cnt + cq, wr[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    float* out = slab + (int64_t)b * k * D;
    for (int e = threadIdx.x; e < k * DS; e += THREADS) {
        const int cc = e / DS, dd = e - cc * DS;
        out[(int64_t)cc * D + d0 + dd] = tab[e];
    }
    if (s == 0)
        for (int cc = threadIdx.x; cc < k; cc += THREADS) slab_cnt[(int64_t)b * k + cc] = cnt[cc];
}

// out[c][0..D) = sum_b slab[b][c][:], out[c][D] = sum_b slab_cnt[b][c]; fp64, fixed order over b
__global__ __launch_bounds__(256) void kmeans_accum_reduce_kernel(const float* __restrict__ slab,
                                                                  const float* __restrict__ slab_cnt, int nchunk,
                                                                  int k, int D, double* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)k * (D + 1);
    if (e >= total) return;
    const int c = (int)(e / (D + 1)), dd = (int)(e - (int64_t)c * (D + 1));
    double acc = 0.0;
    if (dd < D) {
        for (int b = 0; b < nchunk; ++b) acc += (double)slab[((int64_t)b * k + c) * D + dd];
    } else {
        for (int b = 0; b < nchunk; ++b) acc += (double)slab_cnt[(int64_t)b * k + c];
    }
    out[e] = acc;
}

}  // namespace

extern "C" {

// max k for a feature width D (the LDS table of one dim slice must fit the 160 KiB LDS)
int alink_kmeans_accum_kmax(int D) { return D == 64 ? 512 : 256; }

// slab: nchunk * k * D floats, slab_cnt: nchunk * k floats, out: k * (D + 1) doubles.  idx int32 [N] in [0, k)
// (other values are skipped), w nullable fp32 [N].  D == 64 or D % 128 == 0, D <= 1024.  Returns 0 or an error.
int alink_kmeans_accum_bf16(const void* X, int64_t N, int D, const int* idx, const float* w, int k, int nchunk,
                            float* slab, float* slab_cnt, double* out, void* stream) {
    if (N <= 0 || !(D == 64 || (D % 128 == 0 && D <= 1024)) || k < 1 || k > alink_kmeans_accum_kmax(D) ||
        nchunk < 1)
        return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t per = (N + nchunk - 1) / nchunk;
    static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once per kernel
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kmeans_accum_kernel<64>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (512 * 64 + 512) * 4) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(kmeans_accum_kernel<128>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (256 * 128 + 256) * 4) != hipSuccess)
            return 3;
        attr_set = true;
    }
    if (D == 64) {
        const size_t lds = (size_t)(k * 64 + k) * sizeof(float);
        hipLaunchKernelGGL(kmeans_accum_kernel<64>, dim3(nchunk, 1), dim3(THREADS), lds, st, (const __bf16*)X, N, D,
                           idx, w, k, per, slab, slab_cnt);
    } else {
        const size_t lds = (size_t)(k * 128 + k) * sizeof(float);
        hipLaunchKernelGGL(kmeans_accum_kernel<128>, dim3(nchunk, D / 128), dim3(THREADS), lds, st,
                           (const __bf16*)X, N, D, idx, w, k, per, slab, slab_cnt);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    const int64_t total = (int64_t)k * (D + 1);
    hipLaunchKernelGGL(kmeans_accum_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, slab,
                       slab_cnt, nchunk, k, D, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
