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
// keeps its slice of the k x DS fp32 partial sums in LDS (k <= 256 at DS = 128 -> 145 KiB, k <= 512 at DS = 64),
// 8 waves walk the chunk's rows: every wave instruction loads 1 KiB = DS/8 lanes x 16 B per row, 64/(DS/8) rows,
// 8 such loads in flight per wave (64 KiB per CU: the first version, one 256-B row per wave instruction and 4 in
// flight, was latency-bound at 0.4 TB/s), then ds_add_f32 into row idx[r] of the LDS table with the table
// columns permuted (lane l's element j -> column j*DS/8 + l) so consecutive lanes hit consecutive banks.  At the end
// the table goes to slab[b][c][D] (fp32) and a fixed-order fp64 reduction over chunks (kmeans_accum_reduce)
// forms [k][D+1].  Counts of unweighted rows are exact (integers < 2^24 per chunk); the fp32 sums inside a chunk
// depend on the LDS atomic order (rounding-level run-to-run differences, unlike v7's MFMA path).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int THREADS = 512;
constexpr int NW = THREADS / 64;
constexpr int U = 8;                  // 1-KiB wave loads in flight per wave (8 KiB / wave, 64 KiB / CU)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS table row stride RS = DS + 16 (DS = 128: the 2 rows a 32-lane half touches per ds_add_f32 sit in different
// bank halves when their centroid ids differ in parity) or DS + 8 (DS = 64: 4 rows per half, bank offsets 8c mod 32)
template <int DS>
struct Tab {
    static constexpr int RS = DS == 64 ? DS + 8 : DS + 16;
    static constexpr int LPR = DS / 8;              // lanes per row: each lane loads 8 bf16 (16 B)
    static constexpr int RPI = 64 / LPR;            // rows per wave instruction (4 at DS=128, 8 at DS=64)
};

template <int DS>
__global__ __launch_bounds__(THREADS) void kmeans_accum_kernel(const __bf16* __restrict__ X, int64_t N, int D,
                                                               const int* __restrict__ idx,
                                                               const float* __restrict__ w, int k,
                                                               int64_t rows_per_chunk, float* __restrict__ slab,
                                                               float* __restrict__ slab_cnt) {
    using T = Tab<DS>;
    extern __shared__ float tab[];          // [k][RS] then cnt[k]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x, s = blockIdx.y;
    const int d0 = s * DS;
    float* cnt = tab + k * T::RS;
    for (int e = threadIdx.x; e < k * T::RS + k; e += THREADS) tab[e] = 0.f;
    __syncthreads();
    const int64_t r_lo = (int64_t)b * rows_per_chunk;
    const int64_t r_hi = r_lo + rows_per_chunk < N ? r_lo + rows_per_chunk : N;
    const int sub = lane / T::LPR;          // which of the RPI rows of an instruction this lane serves
    const int l = lane % T::LPR;            // 16-B column chunk of that row
    const bool do_cnt = s == 0 && l == 0;
    constexpr int ROWS_PER_ITER = NW * U * T::RPI;
    for (int64_t base = r_lo + (int64_t)wave * U * T::RPI; base < r_hi; base += ROWS_PER_ITER) {
        f32x4 lo[U], hi[U];
        int c[U];
        float wr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = base + u * T::RPI + sub;
            const bool ok = r < r_hi;
            c[u] = ok ? idx[r] : -1;
            wr[u] = ok ? (w != nullptr ? w[r] : 1.f) : 0.f;
            const uint4 v = *reinterpret_cast<const uint4*>(X + (ok ? r : r_lo) * D + d0 + 8 * l);
            lo[u] = f32x4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xFFFF0000u),
                          __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xFFFF0000u)};
            hi[u] = f32x4{__uint_as_float(v.z << 16), __uint_as_float(v.z & 0xFFFF0000u),
                          __uint_as_float(v.w << 16), __uint_as_float(v.w & 0xFFFF0000u)};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (c[u] < 0 || c[u] >= k) continue;
            // table column of element j of this lane's chunk: j * LPR + l (consecutive lanes -> consecutive banks)
            float* row = tab + c[u] * T::RS + l;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                __hip_atomic_fetch_add(row + j * T::LPR, wr[u] * lo[u][j], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(row + (j + 4) * T::LPR, wr[u] * hi[u][j], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (do_cnt) __hip_atomic_fetch_add(cnt + c[u], wr[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    float* out = slab + (int64_t)b * k * D;
    for (int e = threadIdx.x; e < k * DS; e += THREADS) {
        const int cc = e / DS, dd = e - cc * DS;        // dd = 8 * l + j  <->  table column j * LPR + l
        out[(int64_t)cc * D + d0 + dd] = tab[cc * T::RS + (dd & 7) * T::LPR + (dd >> 3)];
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
int alink_kmeans_accum_kmax(int D) { return D == 64 ? 512 : 256; }   // (k * (RS + 1)) * 4 B <= 160 KiB

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
                                hipFuncAttributeMaxDynamicSharedMemorySize, (512 * 72 + 512) * 4) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(kmeans_accum_kernel<128>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (256 * 144 + 256) * 4) != hipSuccess)
            return 3;
        attr_set = true;
    }
    if (D == 64) {
        const size_t lds = (size_t)(k * Tab<64>::RS + k) * sizeof(float);
        hipLaunchKernelGGL(kmeans_accum_kernel<64>, dim3(nchunk, 1), dim3(THREADS), lds, st, (const __bf16*)X, N, D,
                           idx, w, k, per, slab, slab_cnt);
    } else {
        const size_t lds = (size_t)(k * Tab<128>::RS + k) * sizeof(float);
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
