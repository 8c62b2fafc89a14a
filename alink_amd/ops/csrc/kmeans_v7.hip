// KMeans fused assign + accumulate, v7 (gfx950 / MI355X): role-split waves on 16x16x32 MFMA.
//
// One Lloyd superstep over this rank's rows (reference: KMeansAssignCluster.calc -> KMeansUtil.updateSumMatrix,
// A/operator/common/clustering/kmeans/KMeansUtil.java:60-85) in ONE persistent launch, one 512-thread
// workgroup per CU, each workgroup streaming a contiguous run of 64-row tiles HBM -> LDS with LDS-DMA
// (buffer_load ... lds, 5-6 tiles = 80-96 KiB in flight, Plan<KB>).  The 8 waves split by ROLE so every SIMD
// pairs a VALU-heavy wave with an MFMA-heavy one (the waves of a workgroup land on the 4 SIMDs round-robin):
//
//   distance waves 0..3 (tile i):   rows 16w..16w+15 of the tile
//     S^T[c][r] = C[c][:] . X[r][:]  on v_mfma_f32_16x16x32_bf16, the C operand starts at -|c|^2/2, so
//     argmax_c S == argmin_c |x - c|^2; centroid fragments (k padded to 16, not 32 or 128) stay in VGPRs;
//     argmax in registers (centroid id packed into the 7 low mantissa bits, v_max3), two lane swaps;
//     each row then sets ONE bf16 1.0 in the one-hot image Onehot[c][r] (ds_write_b16) and bumps count[c]
//     (ds_add_u32); two tiles later the same lane clears its entry again (no buffer-wide zeroing).
//   accumulate waves 4..7 (tile i-1): dims 32a..32a+31
//     Sum[c][d] += Onehot[c][rows] . X[rows][d] on the same MFMA: A fragments are plain ds_read_b128 of the
//     one-hot image, B fragments ds_read_b64_tr_b16 transposed reads of the SAME X tile image.
//
// One s_barrier per tile.  Every LDS image is bank-conflict-free for its reads (tools/lds_bank_check.py):
// X tile rows are 256 B with the 16-B chunk XOR (row&3)<<2 | (row>>2)&3 (applied to the DMA source
// address), distance reads take dim chunk s + 4*(lane>>4) at k-step s (any dim permutation is exact as long
// as C uses the same one), one-hot rows (128 B) XOR their 16-B chunk with (c>>1)&7.
// End: accumulate waves write fp32 partial sums and the counts to the per-workgroup slab; the fixed-order
// fp64 slab reduction in kmeans.hip makes the [k][D+1] buffer deterministic.
//
// Contract (checked by the host wrapper before launch): D == 128, 1 <= k <= 128, X row-major bf16 [N][128]
// 16-B aligned, C padded [128][128] bf16 (zero rows past k), ninit[128] = -|c|^2/2 (-3e38 past k).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kmeans_tile.h"

namespace {

using namespace kmtile;

// LDS plan per centroid-block count KB: double-buffered one-hot image [16*KB c][64 rows] bf16, u32 count[128],
// and as deep an X ring as the rest of the 160 KiB allows (6 tiles in flight for k <= 112, 5 for k <= 128;
// measured 6.37 -> 6.01 ms at k=100 against the 4-deep ring, profiles/kmeans_r2_session4.txt)
template <int KB>
struct Plan {
    static constexpr int OHB = 16 * KB * TR * 2;
    static constexpr int NBUF_FIT = (LDS_CAP - 2 * OHB - 128 * 4) / TILE;
    static constexpr int NBUF = NBUF_FIT > 8 ? 8 : NBUF_FIT;   // X ring slots: tile i, i-1, AHEAD in flight
    static constexpr int AHEAD = NBUF - 2;
    static constexpr int OFF_OH = NBUF * TILE;
    static constexpr int OFF_CNT = OFF_OH + 2 * OHB;
    static constexpr int LDS_BYTES = OFF_CNT + 128 * 4;
    static_assert(LDS_BYTES <= LDS_CAP && AHEAD >= 3 && AHEAD <= 6, "LDS plan");
};

enum Mode { FULL = 0, LOAD_ONLY = 1, COMPUTE_ONLY = 2 };

// wait until this wave's loads of the tile `younger` tiles before the newest one issued have landed
__device__ __forceinline__ void wait_tile(int younger) {
    if (younger >= 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (younger == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

template <int KB, int MODE, int VAR>
__global__ __launch_bounds__(512) void kmeans_v7_kernel(const __bf16* __restrict__ Xp, int64_t N,
                                                        const __bf16* __restrict__ Cp,
                                                        const float* __restrict__ ninit, float* __restrict__ slab,
                                                        float* __restrict__ slab_cnt, int* __restrict__ assign_out,
                                                        int64_t ntiles, int64_t per) {
    using PL = Plan<KB>;
    constexpr int NBUF = PL::NBUF, AHEAD = PL::AHEAD, OHB = PL::OHB, OFF_OH = PL::OFF_OH, OFF_CNT = PL::OFF_CNT;
    // VAR 0: all 8 waves stage 2 pieces per tile.  VAR 1 (default): the accumulate waves stage all 16 pieces
    // (4 each), so the distance waves — the critical role — carry no LDS-DMA issue cost and no vmcnt waits.
    // (Measured and dropped, profiles/kmeans_r2_session5.txt: an L2 touch of tile i+AHEAD+3, s_setprio on the
    // distance waves, a pairwise-tree argmax, reading tile i+1's distance fragments after barrier i.)
    constexpr bool ACC_DMA = VAR >= 1;
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
        // VAR 0: pieces i < 2 of 8 KiB halves over 512 threads; ACC_DMA: pieces i < 4 of 4 KiB over 256 threads
        const int p = ACC_DMA ? i * 4096 + (tid & 255) * 16 : (i & 1) * 8192 + tid * 16;
        const int row = p >> 8;
        const int chl = ((p >> 4) & 15) ^ xsw(row);
        voff[i] = (uint32_t)(row * ROWB + chl * 16);
    }
    const bool dma_wave = !ACC_DMA || wave >= 4;
    auto stage_tile = [&](int slot, int64_t t) {
        if constexpr (ACC_DMA) stage_np<4>(lds, slot, X, (tbase + t) * TR, N, voff, wave - 4);
        else stage(lds, slot, X, (tbase + t) * TR, N, *reinterpret_cast<const uint32_t(*)[2]>(voff), wave);
    };
    if (MODE != COMPUTE_ONLY && dma_wave)
        for (int s = 0; s < AHEAD; ++s)
            if (s < my_ntiles) stage_tile(s, s);
    {
        for (int e = tid * 16; e < 2 * OHB + 128 * 4; e += 512 * 16)
            *reinterpret_cast<f32x4*>(lds + OFF_OH + e) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    uint32_t* cnt = reinterpret_cast<uint32_t*>(lds + OFF_CNT);

    // per-iteration prologue shared by both roles: tile i has landed (own loads + barrier), refill the ring
    auto pre = [&](int64_t i) {
        if (MODE != COMPUTE_ONLY && dma_wave) {
            if (i < my_ntiles) {
                const int64_t younger = my_ntiles - 1 - i;
                const int y = younger < AHEAD - 1 ? (int)younger : AHEAD - 1;
                if constexpr (ACC_DMA) wait_tile4(y);
                else wait_tile(y);
            }
        }
        barrier_lds();
        if (MODE != COMPUTE_ONLY && dma_wave && i + AHEAD < my_ntiles)
            stage_tile((int)((i + AHEAD) % NBUF), i + AHEAD);
    };

    if (wave < 4) {
        // ------------------------------ distance / argmax role ------------------------------
        const int myrow = 16 * wave + li;
        bf16x8 cf[KB][4];
        f32x4 nin[KB];
#pragma unroll
        for (int b = 0; b < KB; ++b) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
                cf[b][s] = *reinterpret_cast<const bf16x8*>(Cp + (16 * b + li) * D + 8 * (s + 4 * g));
            nin[b] = *reinterpret_cast<const f32x4*>(ninit + 16 * b + 4 * g);
        }
        int xr[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) xr[s] = xoff(myrow, s + 4 * g);
        uint32_t prev1 = NONE, prev2 = NONE;
        for (int64_t i = 0; i <= my_ntiles; ++i) {
            pre(i);
            if (MODE == LOAD_ONLY || i >= my_ntiles) continue;
            const char* xt = lds + (int)(i % NBUF) * TILE;
            f32x4 acc[KB];
#pragma unroll
            for (int b = 0; b < KB; ++b) acc[b] = nin[b];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const bf16x8 xb = *reinterpret_cast<const bf16x8*>(xt + xr[s]);
#pragma unroll
                for (int b = 0; b < KB; ++b)
                    acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cf[b][s], xb, acc[b], 0, 0, 0);
            }
            // all 4*KB MFMAs (KB independent accumulators per k-step) issue before the argmax VALU: without this
            // fence the scheduler interleaves per-block argmax work and serialises the last MFMA of each chain
            __builtin_amdgcn_sched_barrier(0);
            float best = -3.4e38f;
#pragma unroll
            for (int b = 0; b < KB; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) best = pack_max(best, acc[b][r], (uint32_t)(16 * b + 4 * g + r));
            best = fmaxf(best, __shfl_xor(best, 16));
            best = fmaxf(best, __shfl_xor(best, 32));
            if (g == 0) {
                uint16_t* oh = reinterpret_cast<uint16_t*>(lds + OFF_OH + (int)(i & 1) * OHB);
                if (prev2 != NONE) oh[ohoff((int)prev2, myrow) >> 1] = 0;
                const int64_t grow = (tbase + i) * TR + myrow;
                const uint32_t c = __float_as_uint(best) & 127u;
                prev2 = prev1;
                prev1 = NONE;
                if (grow < N) {
                    oh[ohoff((int)c, myrow) >> 1] = 0x3F80;     // bf16 1.0
                    __hip_atomic_fetch_add(cnt + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (assign_out != nullptr) assign_out[grow] = (int)c;
                    prev1 = c;
                }
            }
        }
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
        for (int64_t i = 0; i <= my_ntiles; ++i) {
            pre(i);
            if (MODE == LOAD_ONLY || i == 0) continue;
            const int xt = (int)((i - 1) % NBUF) * TILE;
            const char* oh = lds + OFF_OH + (int)((i - 1) & 1) * OHB;
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

template <int KB, int VAR>
hipError_t launch_kb_var(int mode, dim3 grid, hipStream_t st, const __bf16* X, int64_t N, const __bf16* C,
                         const float* ninit, float* slab, float* slab_cnt, int* assign_out, int64_t ntiles,
                         int64_t per) {
    if (mode == LOAD_ONLY)
        hipLaunchKernelGGL((kmeans_v7_kernel<KB, LOAD_ONLY, VAR>), grid, dim3(512), 0, st, X, N, C, ninit, slab,
                           slab_cnt, assign_out, ntiles, per);
    else if (mode == COMPUTE_ONLY)
        hipLaunchKernelGGL((kmeans_v7_kernel<KB, COMPUTE_ONLY, VAR>), grid, dim3(512), 0, st, X, N, C, ninit,
                           slab, slab_cnt, assign_out, ntiles, per);
    else
        hipLaunchKernelGGL((kmeans_v7_kernel<KB, FULL, VAR>), grid, dim3(512), 0, st, X, N, C, ninit, slab,
                           slab_cnt, assign_out, ntiles, per);
    return hipGetLastError();
}

// mode bits 0-1: 0 full, 1 load only, 2 compute only; bit 4: variant (VAR, see the kernel); the default
// (mode < 16 from the wrapper) is VAR 1: 5.80-5.91 -> 5.50-5.54 ms at k = 100 (profiles/kmeans_r2_session5.txt)
template <int KB>
hipError_t launch_kb(int mode, dim3 grid, hipStream_t st, const __bf16* X, int64_t N, const __bf16* C,
                     const float* ninit, float* slab, float* slab_cnt, int* assign_out, int64_t ntiles,
                     int64_t per) {
    if ((mode >> 4) & 1)
        return launch_kb_var<KB, 1>(mode & 3, grid, st, X, N, C, ninit, slab, slab_cnt, assign_out, ntiles, per);
    return launch_kb_var<KB, 0>(mode & 3, grid, st, X, N, C, ninit, slab, slab_cnt, assign_out, ntiles, per);
}

}  // namespace

extern "C" {

// Fused assign + accumulate (v7).  slab [grid][128][128] f32 and slab_cnt [grid][128] f32 receive one
// partial per workgroup (rows c < 16*ceil(k/16) written); assign_out (nullable) gets the int32 centroid id of
// every row.  mode: 0 full, 1 load pipeline only, 2 compute only (diagnostics; results meaningless).
// Returns 0 or a hipError_t.
int alink_kmeans_assign_accum_bf16_v7(const void* X, int64_t N, const void* C, const float* ninit, int k,
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

// number of workgroups the v7 launch uses for N rows on `grid` CUs (the slab reduction must read exactly those)
int alink_kmeans_v7_grid(int64_t N, int grid) {
    const int64_t ntiles = (N + TR - 1) / TR;
    if (grid > ntiles) grid = (int)ntiles;
    const int64_t per = (ntiles + grid - 1) / grid;
    return (int)((ntiles + per - 1) / per);
}

}  // extern "C"
