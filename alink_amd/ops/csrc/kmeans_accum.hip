// KMeans per-cluster accumulation by a precomputed assignment (gfx950 / MI355X) — the general path.
//
// The fused v7 kernel (kmeans_v7.hip) covers the headline shape (bf16, D = 128, k <= 128, unweighted).  Every
// other bf16 shape — D in {64, 256} (D == 64 or a multiple of 128 up to 1024), k up to 256 (512 at D = 64),
// weighted rows
// (the reference's weighted KMeansAssignCluster, KMeansUtil.updateSumMatrix A/operator/common/clustering/kmeans/
// KMeansUtil.java:60-85) — runs as two passes: the MFMA nearest-centroid kernel (kmeans_nearest.hip) writes
// idx[N], then this kernel forms Sum[c][:] += w_r x_r and Cnt[c] += w_r.
//
// Layout: grid (row chunk b, dim slice s), DS = 64 dims per slice; a 512-thread workgroup keeps its slice of the
// k x DS partial sums of up to 256 centroids (grid z: centroid blocks) in an fp64 LDS table (k * 73 * 8 B <=
// 146 KiB; ds_add_f64 ~9 cycles per wave-instruction on gfx950 against ~193 for ds_add_f32).
// 8 waves walk the chunk's rows: every wave instruction loads 1 KiB = 8 lanes x 16 B per row, 8 rows,
// 8 such loads in flight per wave (64 KiB per CU: the first version, one 256-B row per wave instruction and 4 in
// flight, was latency-bound at 0.4 TB/s), then atomic adds into row idx[r] of the LDS table with the table
// columns permuted (lane l's element j -> column j*DS/8 + l) so consecutive lanes hit consecutive banks.  At the end
// the table goes to slab[b][c][D] (fp32) and a fixed-order fp64 reduction over chunks (kmeans_accum_reduce)
// forms [k][D+1].  Counts of unweighted rows are exact; the partial sums inside a chunk depend on the LDS atomic
// order at the rounding level of the table type (run-to-run differences, unlike v7's MFMA path).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kmeans_tile.h"

namespace {

constexpr int THREADS = 512;
constexpr int NW = THREADS / 64;
constexpr int U = 8;                  // 1-KiB wave loads in flight per wave (8 KiB / wave, 64 KiB / CU)
constexpr int KBLK = 256;             // centroids per fp64 LDS table (k * 73 * 8 B <= 146 KiB)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS table row stride RS = DS + 8 elements at DS = 64 (rows of one wave instruction land on different banks);
// DS + 16 at DS = 128 (no longer launched)
template <int DS>
struct Tab {
    static constexpr int RS = DS == 64 ? DS + 8 : DS + 16;
    static constexpr int LPR = DS / 8;              // lanes per row: each lane loads 8 bf16 (16 B)
    static constexpr int RPI = 64 / LPR;            // rows per wave instruction (4 at DS=128, 8 at DS=64)
};

// AT = the LDS table type.  double (k <= 256, DS = 64): measured on gfx950, one wave-instruction of ds_add_f64 costs
// ~9 cycles against ~193 for ds_add_f32 (profiles/gbdt_r3.txt, LDS atomic probe), so the fp64 table is both the
// faster and the more accurate one; the products w * x are formed exactly in fp64.  float: k up to 512 at D = 64.
// TIn = the row type: __bf16 (one 16-B load = 8 elements per lane) or float (two 16-B loads per lane, the same
// 8-element chunk per lane and the same table layout)
template <int DS, typename AT, typename TIn = __bf16>
__global__ __launch_bounds__(THREADS) void kmeans_accum_kernel(const TIn* __restrict__ X, int64_t N, int D,
                                                               const int* __restrict__ idx,
                                                               const float* __restrict__ w, int k_total,
                                                               int64_t rows_per_chunk, float* __restrict__ slab,
                                                               float* __restrict__ slab_cnt) {
    using T = Tab<DS>;
    // blockIdx.z = centroid block: this workgroup's table holds centroids [c_base, c_base + k) only
    const int c_base = (int)blockIdx.z * KBLK;
    const int k = k_total - c_base < KBLK ? k_total - c_base : KBLK;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    AT* tab = reinterpret_cast<AT*>(lds_raw);   // [k][RS] then cnt[k]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x, s = blockIdx.y;
    const int d0 = s * DS;
    AT* cnt = tab + k * T::RS;
    for (int e = threadIdx.x; e < k * T::RS + k; e += THREADS) tab[e] = (AT)0;
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
            c[u] = ok ? idx[r] - c_base : -1;
            wr[u] = ok ? (w != nullptr ? w[r] : 1.f) : 0.f;
            if constexpr (sizeof(TIn) == 2) {
                const uint4 v = *reinterpret_cast<const uint4*>(X + (ok ? r : r_lo) * D + d0 + 8 * l);
                lo[u] = f32x4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xFFFF0000u),
                              __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xFFFF0000u)};
                hi[u] = f32x4{__uint_as_float(v.z << 16), __uint_as_float(v.z & 0xFFFF0000u),
                              __uint_as_float(v.w << 16), __uint_as_float(v.w & 0xFFFF0000u)};
            } else {
                const f32x4* p = reinterpret_cast<const f32x4*>(X + (ok ? r : r_lo) * D + d0 + 8 * l);
                lo[u] = p[0];
                hi[u] = p[1];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (c[u] < 0 || c[u] >= k) continue;
            // table column of element j of this lane's chunk: j * LPR + l (consecutive lanes -> consecutive banks)
            AT* row = tab + c[u] * T::RS + l;
            const AT wa = (AT)wr[u];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                __hip_atomic_fetch_add(row + j * T::LPR, wa * (AT)lo[u][j], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(row + (j + 4) * T::LPR, wa * (AT)hi[u][j], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (do_cnt) __hip_atomic_fetch_add(cnt + c[u], wa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    float* out = slab + ((int64_t)b * k_total + c_base) * D;
    for (int e = threadIdx.x; e < k * DS; e += THREADS) {
        const int cc = e / DS, dd = e - cc * DS;        // dd = 8 * l + j  <->  table column j * LPR + l
        out[(int64_t)cc * D + d0 + dd] = (float)tab[cc * T::RS + (dd & 7) * T::LPR + (dd >> 3)];
    }
    if (s == 0)
        for (int cc = threadIdx.x; cc < k; cc += THREADS) slab_cnt[(int64_t)b * k_total + c_base + cc] = (float)cnt[cc];
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

// ---------------------------------------------------------------------------------------------------------------
// MFMA accumulate-by-index (D = 128, k <= 256, unweighted): the v7 kernel's one-hot GEMM role fed by idx instead
// of a distance pass.  512 threads: waves 0-3 turn the ids of their 16 rows of every 64-row tile into the
// double-buffered bf16 one-hot image Onehot[c][row] (ids prefetched two tiles ahead; an entry is cleared by the
// same lane two tiles later) and bump count[c]; waves 4-7 stage the LDS-DMA tile ring (4 pieces each) and run
// Sum[c][32a..32a+31] += Onehot[c][rows] . X[rows][..] on v_mfma_f32_16x16x32_bf16 with transposed ds_read_tr16
// B fragments — 2*KB*2 MFMAs per tile per wave instead of one LDS float atomic per (row, dim).
// Output: slab [grid][k][128] fp32, slab_cnt [grid][k] -> kmeans_accum_reduce_kernel (fixed-order fp64).
// ---------------------------------------------------------------------------------------------------------------
template <int KB>
struct AccPlan {
    static constexpr int OHB = 16 * KB * kmtile::TR * 2;
    static constexpr int NBUF_FIT = (kmtile::LDS_CAP - 2 * OHB - 256 * 4) / kmtile::TILE;
    static constexpr int NBUF = NBUF_FIT > 8 ? 8 : NBUF_FIT;
    static constexpr int AHEAD = NBUF - 2;
    static constexpr int OFF_OH = NBUF * kmtile::TILE;
    static constexpr int OFF_CNT = OFF_OH + 2 * OHB;
    static constexpr int LDS_BYTES = OFF_CNT + 256 * 4;
    static_assert(LDS_BYTES <= kmtile::LDS_CAP && AHEAD >= 3 && AHEAD <= 6, "LDS plan");
};

__device__ __forceinline__ void wait_tile4_acc(int younger) { kmtile::wait_tile4(younger); }

template <int KB>
__global__ __launch_bounds__(512) void kmeans_accum_mfma_kernel(const __bf16* __restrict__ Xp, int64_t N,
                                                                const int* __restrict__ idx, int k,
                                                                float* __restrict__ slab,
                                                                float* __restrict__ slab_cnt, int64_t ntiles,
                                                                int64_t per) {
    using namespace kmtile;
    using PL = AccPlan<KB>;
    constexpr int NBUF = PL::NBUF, AHEAD = PL::AHEAD, OHB = PL::OHB, OFF_OH = PL::OFF_OH, OFF_CNT = PL::OFF_CNT;
    __shared__ __attribute__((aligned(16))) char lds[PL::LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4;
    const int li = lane & 15;
    const char* X = reinterpret_cast<const char*>(Xp);
    const int64_t tbase = (int64_t)blockIdx.x * per;
    const int64_t my_ntiles = ntiles > tbase ? (ntiles - tbase < per ? ntiles - tbase : per) : 0;
    uint32_t voff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = i * 4096 + (tid & 255) * 16;
        const int row = p >> 8;
        const int chl = ((p >> 4) & 15) ^ xsw(row);
        voff[i] = (uint32_t)(row * ROWB + chl * 16);
    }
    const bool dma_wave = wave >= 4;
    if (dma_wave)
        for (int s = 0; s < AHEAD; ++s)
            if (s < my_ntiles) stage_np<4>(lds, s, X, (tbase + s) * TR, N, voff, wave - 4);
    for (int e = tid * 16; e < 2 * OHB + 256 * 4; e += 512 * 16)
        *reinterpret_cast<f32x4*>(lds + OFF_OH + e) = f32x4{0.f, 0.f, 0.f, 0.f};
    uint32_t* cnt = reinterpret_cast<uint32_t*>(lds + OFF_CNT);
    auto pre = [&](int64_t i) {
        if (dma_wave && i < my_ntiles) {
            const int64_t younger = my_ntiles - 1 - i;
            wait_tile4_acc(younger < AHEAD - 1 ? (int)younger : AHEAD - 1);
        }
        barrier_lds();
        if (dma_wave && i + AHEAD < my_ntiles)
            stage_np<4>(lds, (int)((i + AHEAD) % NBUF), X, (tbase + i + AHEAD) * TR, N, voff, wave - 4);
    };
    if (wave < 4) {
        // ------------------------------ index role ------------------------------
        const int myrow = 16 * wave + li;
        auto load_id = [&](int64_t t) -> int {
            const int64_t grow = (tbase + t) * TR + myrow;
            return (g == 0 && t < my_ntiles && grow < N) ? idx[grow] : -1;
        };
        int q0 = load_id(0), q1 = load_id(1);
        uint32_t prev1 = NONE, prev2 = NONE;
        for (int64_t i = 0; i <= my_ntiles; ++i) {
            pre(i);
            if (i >= my_ntiles) continue;
            const int c = q0;
            q0 = q1;
            q1 = load_id(i + 2);
            if (g == 0) {
                uint16_t* oh = reinterpret_cast<uint16_t*>(lds + OFF_OH + (int)(i & 1) * OHB);
                if (prev2 != NONE) oh[ohoff((int)prev2, myrow) >> 1] = 0;
                prev2 = prev1;
                prev1 = NONE;
                if (c >= 0 && c < k) {
                    oh[ohoff(c, myrow) >> 1] = 0x3F80;     // bf16 1.0
                    __hip_atomic_fetch_add(cnt + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    prev1 = (uint32_t)c;
                }
            }
        }
        barrier_lds();
    } else {
        // ------------------------------ one-hot accumulate role (as kmeans_v7.hip) ------------------------------
        const int a = wave - 4;
        const uint32_t lbase = (uint32_t)(uintptr_t)(LDS_AS void*)lds;
        int trl[2][2], trh[2][2];
        {
            const int q = li >> 2, p = li & 3;
#pragma unroll
            for (int d = 0; d < 2; ++d)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int ch = 2 * (2 * a + d) + (p >> 1);
                    trl[d][s2] = xoff(32 * s2 + 8 * g + q, ch) + 8 * (p & 1);
                    trh[d][s2] = xoff(32 * s2 + 8 * g + q + 4, ch) + 8 * (p & 1);
                }
        }
        f32x4 sums[KB][2];
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int d = 0; d < 2; ++d) sums[b][d] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int64_t i = 0; i <= my_ntiles; ++i) {
            pre(i);
            if (i == 0) continue;
            const int xt = (int)((i - 1) % NBUF) * TILE;
            const char* oh = lds + OFF_OH + (int)((i - 1) & 1) * OHB;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                bf16x8 bx[2];
#pragma unroll
                for (int d = 0; d < 2; ++d) {
                    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (LDS_AS bf16x4*)(uintptr_t)(lbase + xt + trl[d][s2]));
                    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (LDS_AS bf16x4*)(uintptr_t)(lbase + xt + trh[d][s2]));
                    bx[d] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
#pragma unroll
                for (int b = 0; b < KB; ++b) {
                    const int c = 16 * b + li;
                    const bf16x8 oa = *reinterpret_cast<const bf16x8*>(
                        oh + c * (TR * 2) + 16 * ((4 * s2 + g) ^ ((c >> 1) & 7)));
#pragma unroll
                    for (int d = 0; d < 2; ++d)
                        sums[b][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, bx[d], sums[b][d], 0, 0, 0);
                }
            }
        }
        barrier_lds();
        float* S = slab + (int64_t)blockIdx.x * k * D;
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int d = 0; d < 2; ++d)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int c = 16 * b + 4 * g + r;
                    if (c < k) S[(int64_t)c * D + 16 * (2 * a + d) + li] = sums[b][d][r];
                }
    }
    for (int c = tid; c < k; c += 512) slab_cnt[(int64_t)blockIdx.x * k + c] = (float)cnt[c];
}

template <int KB>
void launch_acc_mfma(dim3 grid, hipStream_t st, const __bf16* X, int64_t N, const int* idx, int k, float* slab,
                     float* slab_cnt, int64_t ntiles, int64_t per) {
    hipLaunchKernelGGL(kmeans_accum_mfma_kernel<KB>, grid, dim3(512), 0, st, X, N, idx, k, slab, slab_cnt, ntiles,
                       per);
}

// max k for a feature width D (the LDS table of one dim slice must fit the 160 KiB LDS)
int accum_kmax(int D) { return D == 64 ? 512 : 256; }   // (k * (RS + 1)) * 4 B <= 160 KiB

template <typename TIn>
int accum_launch(const void* X, int64_t N, int D, const int* idx, const float* w, int k, int nchunk,
                 float* slab, float* slab_cnt, double* out, void* stream) {
    if (N <= 0 || !(D == 64 || (D % 128 == 0 && D <= 1024)) || k < 1 || k > accum_kmax(D) ||
        nchunk < 1)
        return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t per = (N + nchunk - 1) / nchunk;
    static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once per kernel (per TIn)
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kmeans_accum_kernel<64, float, TIn>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (KBLK * 72 + KBLK) * 4) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(kmeans_accum_kernel<64, double, TIn>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (KBLK * 72 + KBLK) * 8) != hipSuccess)
            return 3;
        attr_set = true;
    }
    // one workgroup per (row chunk, 64-dim slice, block of <= 256 centroids); k > 256 re-reads the chunk's rows
    // once per centroid block (an fp64 table of 512 centroids would not fit the LDS)
    const int kb = (k + KBLK - 1) / KBLK;
    const int kl = k < KBLK ? k : KBLK;
    static const bool force_f32 = getenv("ALINK_KMEANS_ACC_F32") != nullptr;   // A/B diagnostic (tools/)
    if (!force_f32) {
        const size_t lds = (size_t)(kl * Tab<64>::RS + kl) * sizeof(double);
        hipLaunchKernelGGL((kmeans_accum_kernel<64, double, TIn>), dim3(nchunk, D / 64, kb), dim3(THREADS), lds, st,
                           (const TIn*)X, N, D, idx, w, k, per, slab, slab_cnt);
    } else {
        const size_t lds = (size_t)(kl * Tab<64>::RS + kl) * sizeof(float);
        hipLaunchKernelGGL((kmeans_accum_kernel<64, float, TIn>), dim3(nchunk, D / 64, kb), dim3(THREADS), lds, st,
                           (const TIn*)X, N, D, idx, w, k, per, slab, slab_cnt);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    const int64_t total = (int64_t)k * (D + 1);
    hipLaunchKernelGGL(kmeans_accum_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, slab,
                       slab_cnt, nchunk, k, D, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace

extern "C" {

int alink_kmeans_accum_kmax(int D) { return accum_kmax(D); }

// slab: nchunk * k * D floats, slab_cnt: nchunk * k floats, out: k * (D + 1) doubles.  idx int32 [N] in [0, k)
// (other values are skipped), w nullable fp32 [N].  D == 64 or D % 128 == 0, D <= 1024.  Returns 0 or an error.
int alink_kmeans_accum_bf16(const void* X, int64_t N, int D, const int* idx, const float* w, int k, int nchunk,
                            float* slab, float* slab_cnt, double* out, void* stream) {
    return accum_launch<__bf16>(X, N, D, idx, w, k, nchunk, slab, slab_cnt, out, stream);
}

// the same accumulate-by-index over fp32 rows (KMeans on fp32 feature matrices: the assignment comes from an fp32
// GEMM + argmax, ops/kmeans.assign_accumulate_f32_hip); 16-B aligned rows, same D / k limits
int alink_kmeans_accum_f32(const void* X, int64_t N, int D, const int* idx, const float* w, int k, int nchunk,
                           float* slab, float* slab_cnt, double* out, void* stream) {
    return accum_launch<float>(X, N, D, idx, w, k, nchunk, slab, slab_cnt, out, stream);
}

// MFMA accumulate-by-index for D = 128, k <= 256 (unweighted).  Returns the number of workgroups used through
// the slab layout contract: slab [grid_used][k][128], slab_cnt [grid_used][k] (size them for `grid`).
int alink_kmeans_accum_mfma_bf16(const void* X, int64_t N, const int* idx, int k, int grid, float* slab,
                                 float* slab_cnt, double* out, void* stream) {
    if (N <= 0 || k < 1 || k > 256 || grid <= 0) return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t ntiles = (N + kmtile::TR - 1) / kmtile::TR;
    if (grid > ntiles) grid = (int)ntiles;
    const int64_t per = (ntiles + grid - 1) / grid;
    const int g2 = (int)((ntiles + per - 1) / per);
    const __bf16* Xb = (const __bf16*)X;
    switch ((k + 15) / 16) {
#define ACASE(V) \
        case V: launch_acc_mfma<V>(dim3(g2), st, Xb, N, idx, k, slab, slab_cnt, ntiles, per); break;
        ACASE(1) ACASE(2) ACASE(3) ACASE(4) ACASE(5) ACASE(6) ACASE(7) ACASE(8) ACASE(9) ACASE(10) ACASE(11)
        ACASE(12) ACASE(13) ACASE(14) ACASE(15)
#undef ACASE
        default: launch_acc_mfma<16>(dim3(g2), st, Xb, N, idx, k, slab, slab_cnt, ntiles, per); break;
    }
    if (hipGetLastError() != hipSuccess) return 2;
    const int64_t total = (int64_t)k * 129;
    hipLaunchKernelGGL(kmeans_accum_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, slab,
                       slab_cnt, g2, k, 128, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
