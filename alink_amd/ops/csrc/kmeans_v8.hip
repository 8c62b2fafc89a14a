// KMeans fused assign + accumulate, v8 (gfx950 / MI355X): v7's role-split waves, software-pipelined.
//
// One Lloyd superstep over this rank's rows (reference: KMeansAssignCluster.calc -> KMeansUtil.updateSumMatrix,
// A/operator/common/clustering/kmeans/KMeansUtil.java:60-85) in ONE persistent launch, one 512-thread
// workgroup per CU streaming a contiguous run of 64-row tiles HBM -> LDS with LDS-DMA (buffer_load ... lds).
//
// v7 measured (profiles/kmeans_v7_v8.txt): load pipeline alone 4.08 ms, compute alone 4.15 ms, full 6.2 ms at
// k=100 — per tile the distance wave's argmax / cross-lane reduce / one-hot write ran as a serial TAIL after
// its MFMAs, behind the same barrier as everything else, so every tile paid MFMA time + tail + LDS latency.
// v8 removes the tail from the critical path:
//
//   distance waves 0..3, iteration i: issue the X reads of tile i, then the argmax of tile i-1 (its scores
//     sit in the other accumulator set, MFMAs issued one iteration ago), the cross-lane max via
//     v_permlane32_swap / v_permlane16_swap (VALU, no LDS round trip), the one-hot write and count of tile
//     i-1, and the 16x16x32 MFMAs of tile i — whose results are not waited for until iteration i+1.
//     Two accumulator sets alternate (loop unrolled by two), so the argmax VALU fills MFMA gaps.
//   accumulate waves 4..7, iteration i: Sum[c][d] += Onehot(i-2)[c][rows] . X(i-2)[rows][d] (same MFMA).
//   ring: tiles i-2 .. i+AHEAD live; NBUF = AHEAD + 3 slots (8 for k <= 112, 7 above; one-hot images are
//   sized 16*ceil(k/16) rows so 8 slots fit the 160 KiB LDS).
//
// LDS images are bank-conflict-free for their reads (tools/lds_bank_check.py; same swizzles as v7):
// X tile rows are 256 B with the 16-B chunk XOR (row&3)<<2 | (row>>2)&3 (applied to the DMA source
// address), one-hot rows (128 B) XOR their 16-B chunk with (c>>1)&7.
// End: accumulate waves write fp32 partial sums and the counts to the per-workgroup slab; the fixed-order
// fp64 slab reduction in kmeans.hip makes the [k][D+1] buffer deterministic.
//
// Contract (checked by the host wrapper before launch): D == 128, 1 <= k <= 128, X row-major bf16 [N][128]
// 16-B aligned, C padded [128][128] bf16 (zero rows past k), ninit[128] = -|c|^2/2 (-3e38 past k).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

constexpr int D = 128;
constexpr int ROWB = D * 2;                // 256 B per row
constexpr int TR = 64;                     // rows per tile
constexpr int TILE = TR * ROWB;            // 16 KiB
constexpr uint32_t NONE = 0xFFFFu;

template <int KB>
struct Cfg {
    static constexpr int NBUF = KB <= 7 ? 8 : 7;           // X ring slots
    static constexpr int AHEAD = NBUF - 3;                  // tiles in flight beyond the three being used
    static constexpr int OHB = 16 * KB * TR * 2;            // one-hot image [16*KB c][64 rows] bf16
    static constexpr int OFF_OH = NBUF * TILE;
    static constexpr int OFF_CNT = OFF_OH + 2 * OHB;        // u32 count[128]
    static constexpr int OFF_NIN = OFF_CNT + 128 * 4;       // f32 -|c|^2/2 [16*KB] (MFMA C-operand init)
    static constexpr int LDS_BYTES = OFF_NIN + 16 * KB * 4;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

enum Mode { FULL = 0, LOAD_ONLY = 1, COMPUTE_ONLY = 2 };

__device__ __forceinline__ int xsw(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int xoff(int row, int ch) { return row * ROWB + 16 * (ch ^ xsw(row)); }
__device__ __forceinline__ int ohoff(int c, int row) {
    return c * (TR * 2) + 16 * ((row >> 3) ^ ((c >> 1) & 7)) + 2 * (row & 7);
}

__device__ __forceinline__ void barrier_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// wait until this wave's two loads of the tile that has `younger` newer tiles issued after it have landed
__device__ __forceinline__ void wait_tile(int younger) {
    switch (younger) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    }
}

// stage one 64-row tile: 16 LDS-DMA pieces of 1 KiB, two per wave; rows past N read as zero (buffer bounds)
__device__ __forceinline__ void stage(char* lds, int slot, const char* X, int64_t row0, int64_t N,
                                      const uint32_t (&voff)[2], int wave) {
    const int64_t rem = (N - row0) * ROWB;
    const int nbytes = rem < TILE ? (int)rem : TILE;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(X + row0 * ROWB), (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(LDS_AS void*)(lds + slot * TILE + i * 8192 + wave * 1024));
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %3\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff[i]), "s"(rs), "s"(m0v)
            : "memory");
    }
}

__device__ __forceinline__ float pack_max(float best, float v, uint32_t c) {
    return fmaxf(best, __uint_as_float((__float_as_uint(v) & 0xFFFFFF80u) | c));
}

// max over lanes l, l^16, l^32, l^48 with VALU lane swaps (gfx950)
__device__ __forceinline__ float max4rows(float v) {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float m = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

template <int KB, int MODE>
__global__ __launch_bounds__(512) void kmeans_v8_kernel(const __bf16* __restrict__ Xp, int64_t N,
                                                        const __bf16* __restrict__ Cp,
                                                        const float* __restrict__ ninit, float* __restrict__ slab,
                                                        float* __restrict__ slab_cnt, int* __restrict__ assign_out,
                                                        int64_t ntiles, int64_t per) {
    using CF = Cfg<KB>;
    constexpr int NBUF = CF::NBUF, AHEAD = CF::AHEAD, OHB = CF::OHB;
    __shared__ __attribute__((aligned(16))) char lds[CF::LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4;
    const int li = lane & 15;
    const char* X = reinterpret_cast<const char*>(Xp);
    const int64_t tbase = (int64_t)blockIdx.x * per;
    const int64_t my_ntiles = ntiles > tbase ? (ntiles - tbase < per ? ntiles - tbase : per) : 0;

    uint32_t voff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int p = i * 8192 + tid * 16;      // linear LDS byte this lane's DMA fills
        const int row = p >> 8;
        const int chl = ((p >> 4) & 15) ^ xsw(row);
        voff[i] = (uint32_t)(row * ROWB + chl * 16);
    }
    if (MODE != COMPUTE_ONLY)
        for (int s = 0; s < AHEAD; ++s)
            if (s < my_ntiles) stage(lds, s, X, (tbase + s) * TR, N, voff, wave);
    for (int e = tid * 16; e < 2 * OHB + 128 * 4; e += 512 * 16)
        *reinterpret_cast<f32x4*>(lds + CF::OFF_OH + e) = f32x4{0.f, 0.f, 0.f, 0.f};
    uint32_t* cnt = reinterpret_cast<uint32_t*>(lds + CF::OFF_CNT);
    if (tid < 16 * KB) reinterpret_cast<float*>(lds + CF::OFF_NIN)[tid] = ninit[tid];

    // per-iteration prologue shared by both roles: tile i has landed (own loads + barrier), refill the ring
    auto pre = [&](int64_t i) {
        if (MODE != COMPUTE_ONLY) {
            if (i < my_ntiles) {
                const int64_t younger = my_ntiles - 1 - i;
                wait_tile(younger < AHEAD - 1 ? (int)younger : AHEAD - 1);
            }
        }
        barrier_lds();
        if (MODE != COMPUTE_ONLY && i + AHEAD < my_ntiles)
            stage(lds, (int)((i + AHEAD) % NBUF), X, (tbase + i + AHEAD) * TR, N, voff, wave);
    };
    // iterations 0 .. my_ntiles+1: distance of tile i, argmax/one-hot of tile i-1, accumulate of tile i-2
    const int64_t iters = my_ntiles + 2;

    if (wave < 4) {
        // ------------------------------ distance / argmax role ------------------------------
        const int myrow = 16 * wave + li;
        bf16x8 cf[KB][4];
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int s = 0; s < 4; ++s)
                cf[b][s] = *reinterpret_cast<const bf16x8*>(Cp + (16 * b + li) * D + 8 * (s + 4 * g));
        const f32x4* nin = reinterpret_cast<const f32x4*>(lds + CF::OFF_NIN) + g;   // [b] at nin[4 * b]
        int xr[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) xr[s] = xoff(myrow, s + 4 * g);
        uint32_t prev1 = NONE, prev2 = NONE;
        f32x4 accA[KB], accB[KB];

        // one iteration: `cur` receives tile i's scores (DIST), `old` holds tile i-1's (ARG).  The steady state
        // (both) is one straight-line block so the scheduler can put the argmax VALU in the MFMA gaps.
        auto body = [&](auto dist_c, auto arg_c, int64_t i, f32x4 (&cur)[KB], f32x4 (&old)[KB]) {
            constexpr bool DIST = decltype(dist_c)::value, ARG = decltype(arg_c)::value;
            pre(i);
            if (MODE == LOAD_ONLY) return;
            bf16x8 xb[4];
            if (DIST) {
                const char* xt = lds + (int)(i % NBUF) * TILE;
#pragma unroll
                for (int s = 0; s < 4; ++s) xb[s] = *reinterpret_cast<const bf16x8*>(xt + xr[s]);
#pragma unroll
                for (int b = 0; b < KB; ++b) cur[b] = nin[4 * b];
            }
            if (ARG) {
                const int64_t t = i - 1;
                float best = -__builtin_inff();            // index bits 0: all-NaN rows land on centroid 0
#pragma unroll
                for (int b = 0; b < KB; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) best = pack_max(best, old[b][r], (uint32_t)(16 * b + 4 * g + r));
                best = max4rows(best);
                uint32_t c = __float_as_uint(best) & 127u;
                if (MODE == COMPUTE_ONLY) c &= 15u;           // garbage scores: stay inside the image
                uint16_t* oh = reinterpret_cast<uint16_t*>(lds + CF::OFF_OH + (int)(t & 1) * OHB);
                const int64_t grow = (tbase + t) * TR + myrow;
                const bool valid = grow < N;
                if (g == 0) {
                    if (prev2 != NONE) oh[ohoff((int)prev2, myrow) >> 1] = 0;
                    if (valid) {
                        oh[ohoff((int)c, myrow) >> 1] = 0x3F80;     // bf16 1.0
                        __hip_atomic_fetch_add(cnt + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (assign_out != nullptr) assign_out[grow] = (int)c;
                    }
                }
                prev2 = prev1;
                prev1 = valid ? c : NONE;
            }
            if (DIST) {
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int b = 0; b < KB; ++b)
                        cur[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cf[b][s], xb[s], cur[b], 0, 0, 0);
            }
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        // i = 0: distance only; 1 .. my_ntiles-1: both; my_ntiles: argmax only; my_ntiles+1: barrier only
        body(T_{}, F_{}, 0, accA, accB);
        int64_t i = 1;
        for (; i + 1 < my_ntiles; i += 2) {
            body(T_{}, T_{}, i, accB, accA);
            body(T_{}, T_{}, i + 1, accA, accB);
        }
        if (i < my_ntiles) {
            body(T_{}, T_{}, i, accB, accA);
            body(F_{}, T_{}, i + 1, accA, accB);       // tile my_ntiles-1's scores are in accB
        } else {
            body(F_{}, T_{}, i, accB, accA);           // tile my_ntiles-1's scores are in accA
        }
        body(F_{}, F_{}, my_ntiles + 1, accA, accB);
        barrier_lds();
    } else {
        // ------------------------------ one-hot accumulate role ------------------------------
        const int a = wave - 4;
        const uint32_t lbase = (uint32_t)(uintptr_t)(LDS_AS void*)lds;
        int trl[2][2], trh[2][2];
        {
            const int q = li >> 2, p = li & 3;
#pragma unroll
            for (int d = 0; d < 2; ++d)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int ch = 2 * (2 * a + d) + (p >> 1);
                    trl[d][s] = xoff(32 * s + 8 * g + q, ch) + 8 * (p & 1);
                    trh[d][s] = xoff(32 * s + 8 * g + q + 4, ch) + 8 * (p & 1);
                }
        }
        int oha[KB][2];
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int c = 16 * b + li;
                oha[b][s] = c * (TR * 2) + 16 * ((4 * s + g) ^ ((c >> 1) & 7));
            }
        f32x4 sums[KB][2];
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int d = 0; d < 2; ++d) sums[b][d] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int64_t i = 0; i < iters; ++i) {
            pre(i);
            if (MODE == LOAD_ONLY || i < 2) continue;
            const int64_t t = i - 2;
            const int xt = (int)(t % NBUF) * TILE;
            const char* oh = lds + CF::OFF_OH + (int)(t & 1) * OHB;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 bx[2];
#pragma unroll
                for (int d = 0; d < 2; ++d) {
                    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (LDS_AS bf16x4*)(uintptr_t)(lbase + xt + trl[d][s]));
                    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (LDS_AS bf16x4*)(uintptr_t)(lbase + xt + trh[d][s]));
                    bx[d] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
#pragma unroll
                for (int b = 0; b < KB; ++b) {
                    const bf16x8 oa = *reinterpret_cast<const bf16x8*>(oh + oha[b][s]);
#pragma unroll
                    for (int d = 0; d < 2; ++d)
                        sums[b][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, bx[d], sums[b][d], 0, 0, 0);
                }
            }
        }
        barrier_lds();
        if (MODE != LOAD_ONLY) {
            float* S = slab + (int64_t)blockIdx.x * 128 * D;
#pragma unroll
            for (int b = 0; b < KB; ++b)
#pragma unroll
                for (int d = 0; d < 2; ++d)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        S[(16 * b + 4 * g + r) * D + 16 * (2 * a + d) + li] = sums[b][d][r];
        }
    }
    if (MODE != LOAD_ONLY && tid < 128)
        slab_cnt[(int64_t)blockIdx.x * 128 + tid] = tid < 16 * KB ? (float)cnt[tid] : 0.f;
}

template <int KB>
hipError_t launch_kb(int mode, dim3 grid, hipStream_t st, const __bf16* X, int64_t N, const __bf16* C,
                     const float* ninit, float* slab, float* slab_cnt, int* assign_out, int64_t ntiles,
                     int64_t per) {
    if (mode == LOAD_ONLY)
        hipLaunchKernelGGL((kmeans_v8_kernel<KB, LOAD_ONLY>), grid, dim3(512), 0, st, X, N, C, ninit, slab,
                           slab_cnt, assign_out, ntiles, per);
    else if (mode == COMPUTE_ONLY)
        hipLaunchKernelGGL((kmeans_v8_kernel<KB, COMPUTE_ONLY>), grid, dim3(512), 0, st, X, N, C, ninit, slab,
                           slab_cnt, assign_out, ntiles, per);
    else
        hipLaunchKernelGGL((kmeans_v8_kernel<KB, FULL>), grid, dim3(512), 0, st, X, N, C, ninit, slab, slab_cnt,
                           assign_out, ntiles, per);
    return hipGetLastError();
}

}  // namespace

extern "C" {

// Fused assign + accumulate (v8).  slab [grid][128][128] f32 and slab_cnt [grid][128] f32 receive one
// partial per workgroup (rows c < 16*ceil(k/16) written); assign_out (nullable) gets the int32 centroid id of
// every row.  mode: 0 full, 1 load pipeline only, 2 compute only (diagnostics; results meaningless).
// The workgroup count is alink_kmeans_v7_grid(N, grid) (same tile partition as v7).  Returns 0 or a hipError_t.
int alink_kmeans_assign_accum_bf16_v8(const void* X, int64_t N, const void* C, const float* ninit, int k,
                                      float* slab, float* slab_cnt, int grid, void* stream, int* assign_out,
                                      int mode) {
    if (N <= 0 || k < 1 || k > 128 || grid <= 0) return -1;
    const int KB = (k + 15) / 16;
    const int64_t ntiles = (N + TR - 1) / TR;
    if (grid > ntiles) grid = (int)ntiles;
    const int64_t per = (ntiles + grid - 1) / grid;
    const int g2 = (int)((ntiles + per - 1) / per);   // no workgroup without tiles
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const __bf16* Xb = (const __bf16*)X;
    const __bf16* Cb = (const __bf16*)C;
    hipError_t e;
    switch (KB) {
        case 1: e = launch_kb<1>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
        case 2: e = launch_kb<2>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
        case 3: e = launch_kb<3>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
        case 4: e = launch_kb<4>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
        case 5: e = launch_kb<5>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
        case 6: e = launch_kb<6>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
        case 7: e = launch_kb<7>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
        default: e = launch_kb<8>(mode, dim3(g2), st, Xb, N, Cb, ninit, slab, slab_cnt, assign_out, ntiles, per); break;
    }
    return (int)e;
}

}  // extern "C"
