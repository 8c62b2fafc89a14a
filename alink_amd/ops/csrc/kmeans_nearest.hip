// Nearest-centroid search for k-means|| initialisation and KMeans predict on CDNA4 (gfx950 / MI355X).
//
// Replaces the reference's per-sample distance loop used while seeding (KMeansInitCentroids.java:40-165:
// the cost of every row to the candidate set, then the nearest candidate of every row for the candidate
// weights) and KMeansModelMapper's per-row argmin (KMeansModelMapper.java:25-106).  In PyTorch the same
// work is ~6 elementwise launches over an [N, m] fp32 matrix; here it is ONE pass over X per chunk of
// up to 256 candidates:
//
//   S[r][c] = x_r . c - |c|^2 / 2        (v_mfma_f32_32x32x16_bf16, fp32 accumulate; -|c|^2/2 is the
//                                          accumulator's initial value)
//   best_r  = argmax_c S[r][c]  (== argmin |x_r - c|^2; ties -> lowest index, like torch.argmin)
//   d2_r    = max(|x_r|^2 - 2 best_r, 0)
//
// * one workgroup = 4 waves; a wave owns 32 rows whose bf16 B fragments stay in 4*KS VGPRs while it
//   sweeps every centroid block of the chunk (C chunk staged once per workgroup in LDS, XOR-swizzled so
//   the 32 rows a fragment read touches fall in distinct 16-byte bank groups);
// * RG = 2 (default for D <= 128): a wave takes two 32-row groups per iteration, so each centroid fragment and
//   bias read from LDS feeds two independent MFMA chains;
// * the next iteration's row fragments are loaded while the current ones run their MFMAs;
// * chunks of > 256 candidates are processed by successive launches that merge into (idx, d2) in place
//   (``merge`` = 1), so X is read once per 256 candidates.
//
// Contract (checked by the Python wrapper): D in {64, 128, 256} (KS = D/16 k-steps), X row-major bf16
// [N][D] 16-byte aligned, C row-major bf16 [m][D], cnorm_half[m] = |c|^2/2 in fp32, 1 <= m.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int NB_MAX = 8;    // centroid blocks of 32 per chunk -> 256 candidates
constexpr float kPkNone = -3.4e38f;   // packed-mode initial best (a real or padding score always exceeds it)
constexpr int WAVES = 4;

template <int KS>
__device__ __forceinline__ int cswz(int row, int ch) {
    // ch: 16-byte chunk index within a row (2*KS chunks); XOR with low row bits
    constexpr int NCH = 2 * KS;
    constexpr int MASK = NCH - 1 < 15 ? NCH - 1 : 15;
    return row * (NCH * 16) + 16 * (ch ^ (row & MASK));
}

// packed score for the counts-mode argmax: the lane-local candidate index li (16 * block + r, < 128) replaces the
// low 7 mantissa bits, as 127 - li so equal truncated scores prefer the lower index; one v_max3 then reduces
// three scores at once (the Lloyd kernel's trick, kmeans_v10.hip pack)
__device__ __forceinline__ float pack_li(float v, uint32_t li) {
    return __uint_as_float((__float_as_uint(v) & 0xFFFFFF80u) | (127u - li));
}

__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int KS, int RG, bool PK = false, bool LAG = false>
__global__ __launch_bounds__(256, LAG ? 1 : 2) void kmeans_nearest_kernel(
    const __bf16* __restrict__ X, int64_t N, const __bf16* __restrict__ C, const float* __restrict__ chalf,
    int m, int c0, int* __restrict__ out_idx, float* __restrict__ out_d2, int merge,
    unsigned long long* __restrict__ counts) {
    constexpr int D = 16 * KS;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int nb = (m + 31) >> 5;
    float* lneg = reinterpret_cast<float*>(lds + nb * 32 * D * 2);  // after the staged chunk
    unsigned* lcnt = reinterpret_cast<unsigned*>(lneg + nb * 32);    // counts mode: rows per candidate
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int h = lane >> 5;
    const int l32 = lane & 31;

    // ---- stage the chunk (zero rows beyond m, padding score -inf) ----
    for (int e = tid; e < nb * 32 * 2 * KS; e += 256) {
        const int row = e / (2 * KS), ch = e % (2 * KS);
        uint4 v = {0u, 0u, 0u, 0u};
        if (row < m) v = *reinterpret_cast<const uint4*>(C + (int64_t)row * D + 8 * ch);
        *reinterpret_cast<uint4*>(lds + cswz<KS>(row, ch)) = v;
    }
    for (int e = tid; e < nb * 32; e += 256) {
        lneg[e] = e < m ? -chalf[e] : -3.0e38f;
        lcnt[e] = 0u;
    }
    __syncthreads();

    // a wave owns RG consecutive 32-row groups per iteration: every centroid fragment read from LDS (and every
    // bias read) feeds RG independent MFMA chains
    const int64_t ngroups = (N + 31) >> 5;
    const int64_t nsuper = (ngroups + RG - 1) / RG;
    const int64_t gstride = (int64_t)gridDim.x * WAVES;
    int64_t g = (int64_t)blockIdx.x * WAVES + wave;

    auto load_frags = [&](int64_t sg, bf16x8 (*xf)[KS]) {
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            int64_t r = (sg * RG + q) * 32 + l32;
            r = r < N ? r : N - 1;
            const bf16x8* p = reinterpret_cast<const bf16x8*>(X + r * D + 8 * h);
#pragma unroll
            for (int s = 0; s < KS; ++s) xf[q][s] = p[2 * s];
        }
    };

    // RG <= 2: the next iteration's fragments load while this one computes (double buffer); RG 3 / 4 have no
    // registers for a second set (256 per lane at 2 waves per SIMD) and rely on the other wave of the SIMD instead
    constexpr bool PF = RG <= 2;
    bf16x8 xf[RG][KS], xn[PF ? RG : 1][KS];
    if (PF && g < nsuper) load_frags(g, xf);
    for (; g < nsuper; g += gstride) {
        const int64_t gn = g + gstride;
        if constexpr (PF) {
            if (gn < nsuper) load_frags(gn, xn);
        } else {
            load_frags(g, xf);
        }

        float xx[RG], best[RG];
        int bidx[RG];
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            float a = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float v = (float)xf[q][s][j];
                    a = fmaf(v, v, a);
                }
            xx[q] = a + __shfl_xor(a, 32);
            best[q] = PK ? kPkNone : -3.4e38f;
            bidx[q] = 0x7fffffff;
        }

        // block b's scores: bias init + KS MFMA k-steps per row group
        auto issue = [&](int b, f32x16 (&acc)[RG]) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float bias = lneg[32 * b + (r & 3) + 8 * (r >> 2) + 4 * h];
#pragma unroll
                for (int q = 0; q < RG; ++q) acc[q][r] = bias;
            }
            const int crow = 32 * b + l32;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const bf16x8 cf = *reinterpret_cast<const bf16x8*>(lds + cswz<KS>(crow, 2 * s + h));
#pragma unroll
                for (int q = 0; q < RG; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf, xf[q][s], acc[q], 0, 0, 0);
            }
        };
        // fold block b's scores into the running argmax (blocks in ascending order: ties keep the lowest index)
        auto reduce = [&](int b, const f32x16 (&acc)[RG]) {
            if constexpr (PK) {
                // counts mode: 16 packed scores folded by v_max3 (6 instructions incl. the running best) instead of
                // a compare and two selects per score.  Exact except for scores equal in their top 25 bits
                // (relative 2^-16): such near-ties resolve by index, which only shifts k-means|| candidate weights
#pragma unroll
                for (int q = 0; q < RG; ++q) {
                    float p[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r) p[r] = pack_li(acc[q][r], (uint32_t)(16 * b + r));
                    const float m0 = max3f(p[0], p[1], p[2]), m1 = max3f(p[3], p[4], p[5]);
                    const float m2 = max3f(p[6], p[7], p[8]), m3 = max3f(p[9], p[10], p[11]);
                    const float m4 = max3f(p[12], p[13], p[14]);
                    best[q] = max3f(max3f(m0, m1, m2), max3f(m3, m4, p[15]), best[q]);
                }
            } else {
#pragma unroll
                for (int q = 0; q < RG; ++q)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int c = 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (acc[q][r] > best[q]) {   // c increases with r inside a lane: strict > keeps the lowest
                            best[q] = acc[q][r];
                            bidx[q] = c;
                        }
                    }
            }
        };
        if constexpr (LAG) {
            // lag-1 software pipeline: block b+1's MFMAs are issued before block b's scores are read, so the
            // argmax VALU work never waits on the matrix pipe's result latency (the v10 kernel's interleave)
            f32x16 accA[RG], accB[RG];
            issue(0, accA);
            for (int b = 0; b < nb; b += 2) {
                if (b + 1 < nb) issue(b + 1, accB);
                reduce(b, accA);
                if (b + 2 < nb) issue(b + 2, accA);
                if (b + 1 < nb) reduce(b + 1, accB);
            }
        } else {
            for (int b = 0; b < nb; ++b) {
                f32x16 acc[RG];
                issue(b, acc);
                reduce(b, acc);
            }
        }
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            if constexpr (PK) {
                // decode the lane's winner (the sentinel = every score NaN: counted nowhere), then merge the halves
                const uint32_t bits = __float_as_uint(best[q]);
                if (bits != __float_as_uint(kPkNone)) {
                    const int li = 127 - (int)(bits & 127u), bb = li >> 4, r = li & 15;
                    bidx[q] = 32 * bb + (r & 3) + 8 * (r >> 2) + 4 * h;
                }
            }
            float bq = best[q];
            int iq = bidx[q];
            const float ob = __shfl_xor(bq, 32);
            const int oi = __shfl_xor(iq, 32);
            if (ob > bq || (ob == bq && oi < iq)) {
                bq = ob;
                iq = oi;
            }
            const int64_t row = (g * RG + q) * 32 + l32;
            if (counts != nullptr) {
                // counts mode (one launch holds every candidate): the k-means|| candidate weights, no per-row output
                if (h == 0 && row < N && (unsigned)iq < (unsigned)m) atomicAdd(lcnt + iq, 1u);   // NaN rows: none
            } else if (h == 0 && row < N) {
                const float d2 = fmaxf(xx[q] - 2.f * bq, 0.f);
                const int gi = iq + c0;
                if (merge) {
                    const float prev = out_d2[row];
                    if (d2 < prev) {
                        out_d2[row] = d2;
                        out_idx[row] = gi;
                    }
                } else {
                    out_d2[row] = d2;
                    out_idx[row] = gi;
                }
            }
        }
        if constexpr (PF) {
            if (gn < nsuper) {
#pragma unroll
                for (int q = 0; q < RG; ++q)
#pragma unroll
                    for (int s = 0; s < KS; ++s) xf[q][s] = xn[q][s];
            }
        }
    }
    if (counts != nullptr) {      // integer sums: the same totals in any order
        __syncthreads();
        for (int e = tid; e < m; e += 256)
            if (lcnt[e] != 0u) atomicAdd(counts + e, (unsigned long long)lcnt[e]);
    }
}

template <int KS, int RG, bool PK, bool LAG>
int launch_k(const void* X, int64_t N, const void* C, const float* chalf, int m, int c0, int* idx, float* d2,
             int merge, int grid, hipStream_t st, unsigned long long* counts) {
    const int nb = (m + 31) / 32;
    const size_t lds = (size_t)nb * 32 * (16 * KS) * 2 + (size_t)nb * 32 * 8;
    static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once per kernel
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kmeans_nearest_kernel<KS, RG, PK, LAG>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                NB_MAX * 32 * 16 * KS * 2 + NB_MAX * 32 * 8) != hipSuccess)
            return 3;
        attr_set = true;
    }
    hipLaunchKernelGGL((kmeans_nearest_kernel<KS, RG, PK, LAG>), dim3(grid), dim3(256), lds, st,
                       reinterpret_cast<const __bf16*>(X), N, reinterpret_cast<const __bf16*>(C), chalf, m, c0,
                       idx, d2, merge, counts);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// A/B (off by default): the packed argmax in counts mode (ALINK_KMEANS_COUNTS_PACKED=1).  Measured round 6 at
// 1e8 x 128, 201 candidates: 7.22 -> 7.00 ms (-3 %), with 1229 rows moved between candidates on near-ties -- too
// little for the changed weights, so the exact compare-and-select argmax stays the default
inline bool counts_packed() {
    const char* e = getenv("ALINK_KMEANS_COUNTS_PACKED");
    return e != nullptr && e[0] == '1';
}

// A/B: ALINK_KMEANS_NEAREST_LAG=1 runs the lag-1 MFMA / argmax software pipeline
inline bool nearest_lag() {
    const char* e = getenv("ALINK_KMEANS_NEAREST_LAG");
    return e != nullptr && e[0] == '1';
}

template <int KS, int RG>
int launch(const void* X, int64_t N, const void* C, const float* chalf, int m, int c0, int* idx, float* d2,
           int merge, int grid, hipStream_t st, unsigned long long* counts) {
    const bool pk = counts != nullptr && counts_packed();
    if (nearest_lag())
        return pk ? launch_k<KS, RG, true, true>(X, N, C, chalf, m, c0, idx, d2, merge, grid, st, counts)
                  : launch_k<KS, RG, false, true>(X, N, C, chalf, m, c0, idx, d2, merge, grid, st, counts);
    return pk ? launch_k<KS, RG, true, false>(X, N, C, chalf, m, c0, idx, d2, merge, grid, st, counts)
              : launch_k<KS, RG, false, false>(X, N, C, chalf, m, c0, idx, d2, merge, grid, st, counts);
}

// k-means|| first cost pass (KMeansInitCentroids.java: every row's distance to the first, randomly drawn center):
// a pure streaming pass, so no MFMA tile — lane l of a wave owns 8 dims (16 bytes) of row (l / LPR), LPR = D / 8
// lanes per row, so every load instruction reads 64 x 16 B = 1 KiB of consecutive rows; the center's 8 dims stay in
// the lane's registers.  cost[r] = sqrt(sum_d (x_rd - c_d)^2) in fp64 (the fp32 sum of squared differences:
// no cancellation, unlike the expanded |x|^2 - 2 x.c + |c|^2 form of the nearest kernel).
// wsum != nullptr: wsum[global wave] = the fp64 sum of that wave's costs (lane sums in row order, then a fixed
// xor tree): the k-means|| threshold's total without a second pass over cost[] -- deterministic for a given grid.
template <int D, int U, bool NT>
__global__ __launch_bounds__(256) void kmeans_cost1_kernel(const __bf16* __restrict__ X, int64_t N,
                                                           const __bf16* __restrict__ c, double* __restrict__ cost,
                                                           double* __restrict__ wsum) {
    constexpr int LPR = D / 8;              // lanes per row
    constexpr int RPW = 64 / LPR;           // rows per wave-instruction (U row groups in flight per lane)
    const int lane = threadIdx.x & 63;
    const int piece = lane % LPR;
    const int sub = lane / LPR;
    float cv[8];
    {
        const uint4 cw = *reinterpret_cast<const uint4*>(c + 8 * piece);
        const __bf16* cb = reinterpret_cast<const __bf16*>(&cw);
#pragma unroll
        for (int j = 0; j < 8; ++j) cv[j] = (float)cb[j];
    }
    const int64_t ngroups = (N + RPW - 1) / RPW;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    double lsum = 0.0;
    for (int64_t g0 = w0 * U; g0 < ngroups; g0 += nwaves * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t r = (g0 + u) * RPW + sub;
            r = r < N ? r : N - 1;
            const u32x4* src = reinterpret_cast<const u32x4*>(X + r * D + 8 * piece);
            if constexpr (NT) v[u] = __builtin_nontemporal_load(src);
            else v[u] = *src;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const __bf16* xb = reinterpret_cast<const __bf16*>(&v[u]);
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float dlt = (float)xb[j] - cv[j];
                s = fmaf(dlt, dlt, s);
            }
#pragma unroll
            for (int off = LPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off);
            const int64_t r = (g0 + u) * RPW + sub;
            if (piece == 0 && r < N) {
                // a row with a NaN / inf value costs 0 (never sampled), as in the nearest kernel's clamped form
                const double dv = __builtin_isfinite(s) ? sqrt((double)s) : 0.0;
                if constexpr (NT) __builtin_nontemporal_store(dv, cost + r);
                else cost[r] = dv;
                lsum += dv;
            }
        }
    }
    if (wsum) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) lsum += __shfl_xor(lsum, off);
        if (lane == 0) wsum[w0] = lsum;
    }
}

// k-means|| oversampling draw (KMeansInitCentroids.java: every row is a candidate with probability
// 2k * cost / sum(cost)): row i of this rank is picked when u(first_row + i) < cost[i] * thre, u being the
// counter-based splitmix64 uniform of the GLOBAL row index (models/clustering/kmeans.py _row_uniform, bit for
// bit: the same 64-bit wrapping products and the same double rounding), so every partitioning picks the same
// rows.  Picked local indices go to out[] in arbitrary order (the caller sorts them); *count receives the number
// of picks (it may exceed cap: then only cap are stored and the caller redoes the draw).
__global__ __launch_bounds__(256) void kmeans_par_pick_kernel(const double* __restrict__ cost, int64_t n,
                                                              int64_t first_row, uint64_t key, double thre,
                                                              int64_t* __restrict__ out, int64_t cap,
                                                              unsigned long long* __restrict__ count) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t z = (uint64_t)(first_row + i) * 0x2545F491ull + key;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        const double u = ((double)(z >> 11) + 0.5) * (1.0 / 9007199254740992.0);
        if (u < cost[i] * thre) {
            const unsigned long long pos = atomicAdd(count, 1ull);
            if ((int64_t)pos < cap) out[pos] = i;
        }
    }
}

// The reference seeding rule over the k-means|| candidates (LocalKmeansFunc.sampleInitialCentroids,
// LocalKmeansFunc.java:36-86) in ONE workgroup: picks 1..k-1, each = the first candidate whose cumulative
// weight x cost reaches U[j-1] x total (numpy/torch searchsorted, side left), then cost = min(cost, D[pick]).
// costs and the cumulative sums live in LDS (n <= SEED_NMAX); the prefix sum is ONE sequential fp64 pass in index
// order, as torch.cumsum on the host, so GPU and CPU pick the same candidates.  *mintot receives the smallest total
// seen (<= 0 means some pick had nothing left to sample: the caller redoes the picks on the host).
// idx0 < 0: the first pick is made here too, as the host did it (models/clustering/kmeans.py _local_kmeans: the
// first candidate whose cumulative weight -- one sequential pass, as torch.cumsum on the CPU -- reaches r0 x total),
// so the caller needs no device -> host read before the picks.
// Per pick two barriers: the scan (one lane) and the count of cw < target (its wave) before the first, the cost
// update -- which also forms the next pick's products -- before the second.
constexpr int SEED_NMAX = 4096;
constexpr int SEED_T = 512;

__device__ __forceinline__ double seq_prefix(double* cw, int n) {
    // one lane: the chain of n dependent fp64 adds is the floor; the LDS reads of the next 16 values are issued
    // before the current 16 are summed, so their latency hides behind the chain
    double run = 0.0;
    int i = 0;
    if (n >= 16) {
        double cur[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) cur[u] = cw[u];
        for (; i + 32 <= n; i += 16) {
            double nxt[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) nxt[u] = cw[i + 16 + u];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                run += cur[u];
                cw[i + u] = run;
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            run += cur[u];
            cw[i + u] = run;
        }
        i += 16;
    }
    for (; i < n; ++i) {
        run += cw[i];
        cw[i] = run;
    }
    return run;
}

__global__ __launch_bounds__(SEED_T) void kmeans_seed_ref_kernel(const double* __restrict__ D,
                                                                 const double* __restrict__ w,
                                                                 const double* __restrict__ U, int n, int k, int idx0,
                                                                 double r0, int64_t* __restrict__ chosen,
                                                                 double* __restrict__ mintot,
                                                                 long long* __restrict__ prof) {
    __shared__ double costs[SEED_NMAX];
    __shared__ double cw[SEED_NMAX];
    __shared__ double tot_sh;
    __shared__ int pick_sh;
    const int t = threadIdx.x;
    const int lane = t & 63;
    // prof != nullptr: 100 MHz wall-clock stamps by lane 0 (start, after the L2 warm-up, then per pick 1..8 after
    // the pick and after the cost update)
    auto stamp = [&](int slot) {
        if (prof && t == 0) prof[slot] = (long long)wall_clock64();
    };
    stamp(0);
    // D was written by kernels spread over all XCDs: pull it into this XCD's L2 once (one dword per 128-byte
    // line, all lanes in parallel) instead of paying a far miss on every pick's row
    {
        const unsigned* Dw = reinterpret_cast<const unsigned*>(D);
        const int64_t words = (int64_t)n * n * 2;
        unsigned acc = 0;
        for (int64_t q = (int64_t)t * 32; q < words; q += (int64_t)SEED_T * 32) acc ^= Dw[q];
        if (acc == 0x9E3779B9u && n < 0) chosen[0] = acc;      // never true (n >= 1): keeps the loads
    }
    stamp(1);
    // one pick: lane 0 of wave 0 forms the sequential prefix (the host order), wave 0 counts cw < target
    // (searchsorted side left on the non-decreasing cw) -- no workgroup barrier between the two
    auto pick_from = [&](double u) -> void {
        if (t < 64) {
            if (t == 0) tot_sh = seq_prefix(cw, n);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double target = u * tot_sh;
            int c = 0;
            for (int i = lane; i < n; i += 64) c += cw[i] < target;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
            if (t == 0) pick_sh = c < n - 1 ? c : n - 1;
        }
    };
    if (idx0 < 0) {
        for (int i = t; i < n; i += SEED_T) cw[i] = w[i];
        __syncthreads();
        pick_from(r0);
        __syncthreads();
        idx0 = pick_sh;
    }
    for (int i = t; i < n; i += SEED_T) {
        const double c = D[(int64_t)idx0 * n + i];
        costs[i] = c;
        cw[i] = w[i] * c;
    }
    if (t == 0) chosen[0] = idx0;
    double mt = 1.0 / 0.0;
    __syncthreads();
    for (int j = 1; j < k; ++j) {
        // cumulative weight x cost in exactly the host order (torch.cumsum on the CPU: products rounded first, then
        // one sequential fp64 sum), so the picks equal the host path's bit for bit, ties and near-ties included
        pick_from(U[j - 1]);
        __syncthreads();
        if (j <= 8) stamp(2 * j);
        const double tot = tot_sh;
        mt = tot < mt ? tot : mt;
        const int pick = pick_sh;
        if (t == 0) chosen[j] = pick;
        for (int i = t; i < n; i += SEED_T) {
            const double dv = D[(int64_t)pick * n + i];
            const double cv = dv < costs[i] ? dv : costs[i];
            costs[i] = cv;
            cw[i] = w[i] * cv;
        }
        __syncthreads();
        if (j <= 8) stamp(2 * j + 1);
    }
    if (t == 0) *mintot = mt;
}

// Weighted Lloyd on the k-means|| candidates in ONE workgroup (LocalKmeansFunc.java:88-141; the torch loop of
// models/clustering/kmeans.py _local_kmeans, EUCLIDEAN): every iteration
//   a[i]  = argmin_c sqrt(|(|x_i|^2 + |c|^2) - 2 x_i.c|)   (first index on ties, as torch.argmin)
//   cnt_c = sum of w[i] over a[i] == c, S_c = sum of x_i * w[i] (both in ascending i: run-to-run deterministic)
//   C_c   = S_c / cnt_c where cnt_c > 0 (else unchanged)
// until the assignment stops changing, a cluster is empty (the host refills it from its generator and calls
// again) or max_iter iterations ran.  One CU, so an iteration is bound by fp64 issue and latency:
//   * x.c on the VALU (tile = 8 samples x 64 centroids, below); on gfx950 the f64 MFMA form of the same tiles
//     measured 83 us per iteration against ~40 for this (tools/kmeans_local_bench.py, profiles/kmeans_init_r6.txt);
//   * the per-(sample, 64-centroid tile) winners go through the small global scratch bd / bi and are combined in
//     ascending tile order (strict <: the first index wins);
//   * member counts and members (ascending i) by wave ballots, one wave per cluster; the offsets by one
//     register-carried prefix; cnt_c and S_c by one wave per cluster (lanes over the dims, members in ascending
//     order, 4 rows in flight).
// Centroids live in LDS (rows padded to d + 1 doubles, so the 64 lanes -- 64 centroids -- hit distinct banks),
// weights and the per-sample state too (the caller checks the footprint, local_lloyd_lds, against 160 KiB).
// chosen != nullptr: C starts as the rows X[chosen[c]] (the seeding kernel's picks).  A non-finite sample,
// weight or start centroid: status[3] = 1 and nothing is written (the caller takes the torch path).
// status (fp64 [6]): iterations run, assignment changed in the last one, an empty cluster in the last one,
// non-finite input, *mintot (when given), chosen[0] (when given); live_out[c] = cnt_c > 0 after the last one.
constexpr int LL_T = 1024;
constexpr int LL_RS = 8;

__global__ __launch_bounds__(LL_T) void kmeans_local_lloyd_kernel(
        const double* __restrict__ X, const double* __restrict__ w, int n, int d, int k,
        const int64_t* __restrict__ chosen, double* __restrict__ C, int64_t* __restrict__ assign,
        double* __restrict__ bd, int* __restrict__ bi, int max_iter, const double* __restrict__ mintot,
        double* __restrict__ status, unsigned char* __restrict__ live_out, long long* __restrict__ prof) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int ds = d + 1;
    double* Cs = reinterpret_cast<double*>(lds);             // [k][ds]
    double* cn = Cs + (size_t)k * ds;                         // [k]
    double* cnt = cn + k;                                     // [k]
    double* xn = cnt + k;                                     // [n]
    double* wl = xn + n;                                      // [n]
    int* a = reinterpret_cast<int*>(wl + n);                  // [n]
    int* mem = a + n;                                         // [n] members, cluster-major, ascending i
    int* off = mem + n;                                       // [k + 1]
    __shared__ int flags[5];                                  // [0] non-finite; [1 + 2 * parity] changed / empty
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    constexpr int NW = LL_T / 64;
    // prof != nullptr: lane 0 stamps the 100 MHz wall clock after every barrier (setup; per iteration, up to 8:
    // centroid norms, distances + assignment, member counts, offsets, members + weights, sums)
    auto stamp = [&](int slot) {
        if (prof && t == 0) prof[slot] = (long long)wall_clock64();
    };
    stamp(0);
    if (t < 5) flags[t] = 0;
    __syncthreads();
    int bad = 0;
    for (int q = t; q < n * d; q += LL_T) bad |= !__builtin_isfinite(X[q]);
    for (int q = t; q < n; q += LL_T) {
        const double wq = w[q];
        bad |= !__builtin_isfinite(wq);
        wl[q] = wq;
        a[q] = (int)assign[q];
    }
    for (int q = t; q < k * d; q += LL_T) {
        const int c = q / d, j = q - c * d;
        const double v = chosen ? X[chosen[c] * d + j] : C[q];
        bad |= !__builtin_isfinite(v);
        Cs[c * ds + j] = v;
    }
    for (int i = wv; i < n; i += NW) {                        // |x_i|^2: one wave per sample, fixed order
        double s = 0.0;
        for (int j = lane; j < d; j += 64) {
            const double x = X[(size_t)i * d + j];
            s += x * x;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) xn[i] = s;
    }
    if (bad) atomicOr(&flags[0], 1);
    __syncthreads();
    stamp(1);
    if (flags[0]) {
        if (t == 0) {
            status[0] = 0; status[1] = 0; status[2] = 0; status[3] = 1;
            status[4] = mintot ? *mintot : 0.0;
            status[5] = chosen ? (double)chosen[0] : -1.0;
        }
        return;
    }
    const int CT = (k + 63) / 64;                             // 64-centroid tiles
    const int ntiles = ((n + LL_RS - 1) / LL_RS) * CT;
    int it = 0, changed = 0, empty = 0;
    while (it < max_iter) {
        const int par = 1 + 2 * (it & 1);
        if (t == 0) {
            flags[par] = 0;
            flags[par + 1] = 0;
        }
        for (int c = wv; c < k; c += NW) {                  // |c|^2: one wave per centroid, fixed order
            double s = 0.0;
            for (int j = lane; j < d; j += 64) {
                const double v = Cs[c * ds + j];
                s += v * v;
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            if (lane == 0) cn[c] = s;
        }
        __syncthreads();
        if (it < 8) stamp(2 + it * 6 + 0);
        // x.c on the VALU: a wave tile is LL_RS samples x 64 centroids (lane = centroid); the centroid value comes
        // from LDS, the LL_RS sample values are wave-uniform (scalar) loads, so every LDS read feeds LL_RS fp64 FMAs.
        // The tile's per-sample winner (64-lane argmin) goes to the global scratch bd / bi (L2-resident).
        for (int tile = wv; tile < ntiles; tile += NW) {
            const int sb = tile / CT, ct = tile - sb * CT;
            const int c = ct * 64 + lane;
            const bool cok = c < k;
            const double* crow = Cs + (size_t)(cok ? c : 0) * ds;
            const int i0 = sb * LL_RS;
            const double* xr[LL_RS];
#pragma unroll
            for (int r = 0; r < LL_RS; ++r) xr[r] = X + (size_t)(i0 + r < n ? i0 + r : n - 1) * d;
            double acc[LL_RS];
#pragma unroll
            for (int r = 0; r < LL_RS; ++r) acc[r] = 0.0;
            int j = 0;
            for (; j + 4 <= d; j += 4) {
                double cj[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) cj[u] = crow[j + u];
#pragma unroll
                for (int r = 0; r < LL_RS; ++r)
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc[r] = __builtin_fma(xr[r][j + u], cj[u], acc[r]);
            }
            for (; j < d; ++j) {
                const double cj = crow[j];
#pragma unroll
                for (int r = 0; r < LL_RS; ++r) acc[r] = __builtin_fma(xr[r][j], cj, acc[r]);
            }
#pragma unroll
            for (int r = 0; r < LL_RS; ++r) {
                const int i = i0 + r;
                if (i >= n) break;                              // wave-uniform
                double dist = 1.0 / 0.0;
                int ci = 0x7fffffff;
                if (cok) {
                    dist = __builtin_sqrt(__builtin_fabs((xn[i] + cn[c]) - 2.0 * acc[r]));
                    ci = c;
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const double od = __shfl_xor(dist, o);
                    const int oc = __shfl_xor(ci, o);
                    if (od < dist || (od == dist && oc < ci)) {
                        dist = od;
                        ci = oc;
                    }
                }
                if (lane == 0) {
                    bd[(size_t)i * CT + ct] = dist;
                    bi[(size_t)i * CT + ct] = ci;
                }
            }
        }
        __syncthreads();
        int ch = 0;
        for (int i = t; i < n; i += LL_T) {
            double b = bd[(size_t)i * CT];
            int bc = bi[(size_t)i * CT];
            for (int ct = 1; ct < CT; ++ct) {                // ascending tiles, strict <: the first index wins
                const double o = bd[(size_t)i * CT + ct];
                if (o < b) {
                    b = o;
                    bc = bi[(size_t)i * CT + ct];
                }
            }
            ch |= bc != a[i];
            a[i] = bc;
        }
        if (ch) atomicOr(&flags[par], 1);
        __syncthreads();
        if (it < 8) stamp(2 + it * 6 + 1);
        // member counts: one wave per cluster, 64 samples per ballot
        for (int c = wv; c < k; c += NW) {
            int m = 0;
            for (int b = 0; b < n; b += 64) {
                const int i = b + lane;
                m += __popcll(__ballot(i < n && a[i] == c));
            }
            if (lane == 0) off[c + 1] = m;
        }
        __syncthreads();
        if (it < 8) stamp(2 + it * 6 + 2);
        if (t == 0) {
            int run = 0;
            off[0] = 0;
            for (int c = 1; c <= k; ++c) {
                run += off[c];
                off[c] = run;
            }
        }
        __syncthreads();
        if (it < 8) stamp(2 + it * 6 + 3);
        for (int c = wv; c < k; c += NW) {                  // members in ascending i, by ballot rank
            int p = off[c];
            for (int b = 0; b < n; b += 64) {
                const int i = b + lane;
                const bool mine = i < n && a[i] == c;
                const unsigned long long bal = __ballot(mine);
                if (mine) mem[p + __popcll(bal & ((1ull << lane) - 1ull))] = i;
                p += __popcll(bal);
            }
        }
        __syncthreads();
        if (it < 8) stamp(2 + it * 6 + 4);
        // S_c / cnt_c: one wave per cluster, lanes over the dims, members in ascending order, 4 rows in flight
        int em = 0;
        for (int c = wv; c < k; c += NW) {
            const int m0 = off[c], m1 = off[c + 1];
            double cc = 0.0;                                    // cnt_c: the members' weights in ascending i
            for (int m = m0; m < m1; ++m) cc += wl[mem[m]];
            if (lane == 0) cnt[c] = cc;
            if (!(cc > 0.0)) {
                em = 1;
                continue;
            }
            for (int jg = 0; jg < d; jg += 128) {               // two dims per lane, 4 member rows: 8 loads in flight
                const int ja = jg + lane, jb2 = jg + 64 + lane;
                double sa = 0.0, sb = 0.0;
                for (int m = m0; m < m1; m += 4) {
                    double va[4], vb[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = mem[m + u < m1 ? m + u : m];
                        va[u] = ja < d ? X[(size_t)i * d + ja] : 0.0;
                        vb[u] = jb2 < d ? X[(size_t)i * d + jb2] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (m + u < m1) {
                            const double wi = wl[mem[m + u]];
                            const double pa = va[u] * wi, pb = vb[u] * wi;
                            sa += pa;
                            sb += pb;
                        }
                }
                if (ja < d) Cs[c * ds + ja] = sa / cc;
                if (jb2 < d) Cs[c * ds + jb2] = sb / cc;
            }
        }
        if (em && lane == 0) atomicOr(&flags[par + 1], 1);
        __syncthreads();
        if (it < 8) stamp(2 + it * 6 + 5);
        changed = flags[par];
        empty = flags[par + 1];
        ++it;
        if (!changed || empty) break;                          // uniform: read after the barrier
    }
    for (int q = t; q < k * d; q += LL_T) {
        const int c = q / d, j = q - c * d;
        C[q] = Cs[c * ds + j];
    }
    for (int i = t; i < n; i += LL_T) assign[i] = a[i];
    for (int c = t; c < k; c += LL_T) live_out[c] = it > 0 ? (unsigned char)(cnt[c] > 0.0) : 1;
    if (t == 0) {
        status[0] = it; status[1] = changed; status[2] = empty; status[3] = 0;
        status[4] = mintot ? *mintot : 0.0;
        status[5] = chosen ? (double)chosen[0] : -1.0;
    }
}

size_t local_lloyd_lds(int n, int d, int k) {
    return ((size_t)k * (d + 1) + 2 * (size_t)k + 2 * (size_t)n) * 8 + (2 * (size_t)n + k + 1) * 4;
}

template <int U, bool NT>
int launch_cost1(const __bf16* Xb, int64_t N, int D, const __bf16* cb, double* cost, double* wsum, int grid,
                 hipStream_t st) {
    switch (D) {
        case 64: hipLaunchKernelGGL((kmeans_cost1_kernel<64, U, NT>), dim3(grid), dim3(256), 0, st, Xb, N, cb, cost, wsum); break;
        case 128: hipLaunchKernelGGL((kmeans_cost1_kernel<128, U, NT>), dim3(grid), dim3(256), 0, st, Xb, N, cb, cost, wsum); break;
        case 256: hipLaunchKernelGGL((kmeans_cost1_kernel<256, U, NT>), dim3(grid), dim3(256), 0, st, Xb, N, cb, cost, wsum); break;
        default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace

extern "C" {

// k-means|| first cost pass: cost[r] = |x_r - c| (fp64) for one bf16 center c [D]; D in {64, 128, 256}.
// variant (rows in flight per lane / load policy; profiles/kmeans_init_r5.txt): 0 = 8, non-temporal loads and
// stores; 1 = 8, cached (the default: 4.77 ms at 1e8 x 128, 5.5 TB/s); 2 = 16, non-temporal; 3 = 4, non-temporal
// wsum: nullptr, or [grid * 4] per-wave cost sums (kmeans_cost1_kernel)
int alink_kmeans_cost1_bf16_sum(const void* X, int64_t N, int D, const void* c, double* cost, double* wsum, int grid,
                                int variant, void* stream) {
    if (N <= 0 || grid <= 0) return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const __bf16* Xb = reinterpret_cast<const __bf16*>(X);
    const __bf16* cb = reinterpret_cast<const __bf16*>(c);
    switch (variant) {
        case 0: return launch_cost1<8, true>(Xb, N, D, cb, cost, wsum, grid, st);
        case 1: return launch_cost1<8, false>(Xb, N, D, cb, cost, wsum, grid, st);
        case 2: return launch_cost1<16, true>(Xb, N, D, cb, cost, wsum, grid, st);
        case 3: return launch_cost1<4, true>(Xb, N, D, cb, cost, wsum, grid, st);
        default: return 1;
    }
}

int alink_kmeans_cost1_bf16(const void* X, int64_t N, int D, const void* c, double* cost, int grid, int variant,
                            void* stream) {
    return alink_kmeans_cost1_bf16_sum(X, N, D, c, cost, nullptr, grid, variant, stream);
}

// reference-rule k-means++ picks over n <= 4096 candidates (kmeans_seed_ref_kernel): D [n][n], w [n], U [k-1];
// idx0 < 0: the first pick from r0 (the first candidate whose cumulative weight reaches r0 x total)
int alink_kmeans_seed_ref2(const double* D, const double* w, const double* U, int n, int k, int idx0, double r0,
                           int64_t* chosen, double* mintot, long long* prof, void* stream) {
    if (n < 1 || n > SEED_NMAX || k < 1 || idx0 >= n) return 1;
    hipLaunchKernelGGL(kmeans_seed_ref_kernel, dim3(1), dim3(SEED_T), 0, reinterpret_cast<hipStream_t>(stream), D, w,
                       U, n, k, idx0, r0, chosen, mintot, prof);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

int alink_kmeans_seed_ref(const double* D, const double* w, const double* U, int n, int k, int idx0, int64_t* chosen,
                          double* mintot, void* stream) {
    if (idx0 < 0) return 1;
    return alink_kmeans_seed_ref2(D, w, U, n, k, idx0, 0.0, chosen, mintot, nullptr, stream);
}

// weighted Lloyd on n <= 4096 fp64 candidates X [n][d], weights w [n], k centroids C [k][d] (in/out; taken from
// X[chosen] when chosen != nullptr), assign [n] int64 (in/out, -1 = none); scratch bd fp64 / bi int32
// [n * ceil(k / 64)]; status fp64 [6], live_out uint8 [k] (kmeans_local_lloyd_kernel)
int alink_kmeans_local_lloyd(const double* X, const double* w, int n, int d, int k, const int64_t* chosen, double* C,
                             int64_t* assign, double* bd, int* bi, int max_iter, const double* mintot, double* status,
                             unsigned char* live_out, long long* prof, void* stream) {
    if (n < 1 || n > SEED_NMAX || d < 1 || k < 1 || max_iter < 0) return 1;
    const size_t lds = local_lloyd_lds(n, d, k);
    if (lds > 160 * 1024) return 3;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kmeans_local_lloyd_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return 4;
    hipLaunchKernelGGL(kmeans_local_lloyd_kernel, dim3(1), dim3(LL_T), lds, reinterpret_cast<hipStream_t>(stream), X,
                       w, n, d, k, chosen, C, assign, bd, bi, max_iter, mintot, status, live_out, prof);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// k-means|| oversampling picks of this rank's rows (kmeans_par_pick_kernel); *count must be zero on entry
int alink_kmeans_par_pick(const double* cost, int64_t n, int64_t first_row, int64_t key, double thre, int64_t* out,
                          int64_t cap, void* count, void* stream) {
    if (n < 0 || cap < 0) return 1;
    if (n == 0) return 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(kmeans_par_pick_kernel, dim3((unsigned)blocks), dim3(256), 0, st, cost, n, first_row,
                       (uint64_t)key, thre, out, cap, reinterpret_cast<unsigned long long*>(count));
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// one chunk (m <= 256) of nearest-centroid search; grid = persistent workgroups; rg = 32-row groups per wave
// iteration (1 or 2; 2 needs D <= 128)
// counts != nullptr: no per-row output (out_idx / out_d2 unused, merge must be 0); counts[j] (uint64, zeroed by the
// caller) += rows whose nearest candidate is j — the k-means|| candidate weights of a single-launch candidate set
int alink_kmeans_nearest_bf16_rg(const void* X, int64_t N, int D, const void* C, const float* chalf, int m, int c0,
                                 int* out_idx, float* out_d2, int merge, int grid, int rg, void* counts_v,
                                 void* stream) {
    if (N <= 0 || m <= 0 || m > NB_MAX * 32 || grid <= 0 || rg < 1 || rg > 4 || (rg > 1 && D > 128)) return 1;
    unsigned long long* counts = reinterpret_cast<unsigned long long*>(counts_v);
    if (counts != nullptr && (merge || c0 != 0)) return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (rg == 2) {
        switch (D) {
            case 64: return launch<4, 2>(X, N, C, chalf, m, c0, out_idx, out_d2, merge, grid, st, counts);
            case 128: return launch<8, 2>(X, N, C, chalf, m, c0, out_idx, out_d2, merge, grid, st, counts);
            default: return 1;
        }
    }
    // RG 3 / 4 (D = 128, A/B): each LDS centroid fragment feeds 3 / 4 MFMA chains
    if (rg == 3) return D == 128 ? launch<8, 3>(X, N, C, chalf, m, c0, out_idx, out_d2, merge, grid, st, counts) : 1;
    if (rg == 4) return D == 128 ? launch<8, 4>(X, N, C, chalf, m, c0, out_idx, out_d2, merge, grid, st, counts) : 1;
    switch (D) {
        case 64: return launch<4, 1>(X, N, C, chalf, m, c0, out_idx, out_d2, merge, grid, st, counts);
        case 128: return launch<8, 1>(X, N, C, chalf, m, c0, out_idx, out_d2, merge, grid, st, counts);
        case 256: return launch<16, 1>(X, N, C, chalf, m, c0, out_idx, out_d2, merge, grid, st, counts);
        default: return 1;
    }
}

int alink_kmeans_nearest_bf16(const void* X, int64_t N, int D, const void* C, const float* chalf, int m, int c0,
                              int* out_idx, float* out_d2, int merge, int grid, void* stream) {
    return alink_kmeans_nearest_bf16_rg(X, N, D, C, chalf, m, c0, out_idx, out_d2, merge, grid, 1, nullptr, stream);
}

}  // extern "C"
