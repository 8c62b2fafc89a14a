// Fused KMeans assign + accumulate for CDNA4 (gfx950 / MI355X).
//
// Replaces the reference's per-sample Java loop (KMeansAssignCluster.calc -> KMeansUtil.updateSumMatrix,
// A/operator/common/clustering/kmeans/KMeansUtil.java:60-85, distance via EuclideanDistance gemv
// A/operator/common/distance/EuclideanDistance.java:109-141) with ONE persistent kernel per superstep:
//
//   per 128-row tile (staged HBM -> LDS by global_load_lds, 3-deep ring, swizzled image):
//     1. distance GEMM on MFMA (v_mfma_f32_32x32x16_bf16):  S[c][r] = x_r . c  -  |c|^2 / 2
//        (the -|c|^2/2 term is the accumulator's initial value, so argmax S == argmin ||x - c||^2);
//        wave w owns rows 32w..32w+31, centroid fragments live in registers for the whole kernel;
//     2. argmax over centroids in registers (index packed into the 7 low mantissa bits, v_max_f32);
//     3. one-hot accumulate on MFMA:  Sum[c][d] += Onehot[c][r] . X[r][d]
//        one-hot A fragments come from a 256-entry byte->8xbf16 LUT in LDS indexed by per-centroid row
//        bitmasks (built with ds_or_b32), X^T B fragments from ds_read_b64_tr_b16 on the same LDS image;
//        wave w owns centroid block w (32 centroids x 128 dims, 64 accumulators).
//   end: each workgroup writes its fp32 partial sums + counts (slab); a second kernel reduces slabs in a
//   fixed order in fp64 -> deterministic [k][d+1] buffer that the BSP AllReduce then sums across GPUs.
//
// Contract (checked on the host by the Python wrapper before launch):
//   D == 128, 1 <= k <= 128, X row-major bf16 [N][128] (16-byte aligned), C padded [128][128] bf16
//   (zero rows beyond k), ninit[128] (-|c|^2/2 for c < k, -3e38 for padding).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

constexpr int D = 128;               // feature dims (fast path)
constexpr int TR = 128;              // rows per tile
constexpr int ROWB = D * 2;          // 256 B per row
constexpr int TILE_BYTES = TR * ROWB;  // 32 KiB
constexpr int NSTAGE = 3;            // LDS ring depth (tiles in flight = NSTAGE - 1)
constexpr int GLDS_PER_THREAD = TILE_BYTES / (256 * 16);  // 8

// LDS carve (one __shared__ array: avoids hipcc's extra vmcnt(0) on a second LDS object)
constexpr int OFF_X = 0;
constexpr int OFF_LUT = NSTAGE * TILE_BYTES;          // 256 x 16 B
constexpr int OFF_MASK = OFF_LUT + 256 * 16;          // [2][128 c][4 words]
constexpr int OFF_NINIT = OFF_MASK + 2 * 128 * 4 * 4; // [128] f32
constexpr int LDS_BYTES = OFF_NINIT + 128 * 4;

// swizzled image of a [rows][16 chunks of 16 B] tile (conflict-free for 32x32x16 row reads and
// for ds_read_b64_tr_b16 transposed reads)
__device__ __forceinline__ int xoff(int row, int ch) {
    return row * ROWB + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ void wait_vmcnt_n(int n) {
    // n is one of {0, 8, 16}; immediates must be literal
    if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void barrier_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// stage one 128-row tile (rows >= N are clamped to N-1; their mask bits are never set)
__device__ __forceinline__ void stage_tile(char* lds, int buf, const char* X, int64_t row0, int64_t N,
                                           int tid, int wave) {
    char* dst_base = lds + OFF_X + buf * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < GLDS_PER_THREAD; ++i) {
        const int p = i * 4096 + tid * 16;       // linear LDS byte this lane fills
        const int row = p >> 8;
        const int chp = (p >> 4) & 15;           // physical chunk
        const int chl = chp ^ (((row & 3) << 2) | ((row >> 2) & 3));  // logical chunk stored there
        int64_t grow = row0 + row;
        grow = grow < N ? grow : (N - 1);
        const char* src = X + grow * ROWB + chl * 16;
        // LDS-DMA issued from inline asm: hipcc does not track it, so it does not drain the ring with
        // vmcnt(0) before unrelated LDS accesses; completion is counted by hand (wait_vmcnt_n).
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)LDS_PTR(dst_base + i * 4096 + wave * 1024));
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(m0v)
            : "memory");
    }
}

template <int KB>
__global__ __launch_bounds__(256, 1) void kmeans_assign_accum_kernel(
    const __bf16* __restrict__ Xp, int64_t N, const __bf16* __restrict__ Cp, const float* __restrict__ ninit,
    float* __restrict__ slab, float* __restrict__ slab_cnt, int64_t ntiles) {
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const char* X = reinterpret_cast<const char*>(Xp);

    const int64_t G = gridDim.x;
    const int64_t my_ntiles = (ntiles > (int64_t)blockIdx.x) ? (ntiles - 1 - blockIdx.x) / G + 1 : 0;

    // ---- prologue: start the tile ring before any other setup ----
    for (int s = 0; s < NSTAGE - 1; ++s)
        if (s < my_ntiles) stage_tile(lds, s, X, ((int64_t)blockIdx.x + s * G) * TR, N, tid, wave);

    // LUT: byte -> 8 x bf16 {0, 1.0}; masks cleared; ninit
    {
        uint32_t* lut = reinterpret_cast<uint32_t*>(lds + OFF_LUT);
        for (int e = tid; e < 256 * 4; e += 256) {
            const int ent = e >> 2, pair = e & 3;
            const uint32_t b0 = (ent >> (2 * pair)) & 1, b1 = (ent >> (2 * pair + 1)) & 1;
            lut[e] = (b0 ? 0x3F80u : 0u) | (b1 ? 0x3F800000u : 0u);
        }
        uint32_t* m = reinterpret_cast<uint32_t*>(lds + OFF_MASK);
        for (int e = tid; e < 2 * 128 * 4; e += 256) m[e] = 0u;
        float* ni = reinterpret_cast<float*>(lds + OFF_NINIT);
        if (tid < 128) ni[tid] = ninit[tid];
    }
    // centroid A fragments in registers: cf[b][s] = C[32b + l32][16s + 8h .. +7]
    bf16x8 cf[KB][8];
#pragma unroll
    for (int b = 0; b < KB; ++b)
#pragma unroll
        for (int s = 0; s < 8; ++s)
            cf[b][s] = *reinterpret_cast<const bf16x8*>(Cp + (32 * b + l32) * D + 16 * s + 8 * h);
    // consume the fragments here so hipcc places its load waits before the loop, not at their first
    // (in-loop) use where a per-iteration vmcnt(N<16) would drain the LDS-DMA ring
#pragma unroll
    for (int b = 0; b < KB; ++b)
#pragma unroll
        for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(cf[b][s]));

    f32x16 sacc[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[db][r] = 0.f;
    float cnt = 0.f;

    // make the prologue's non-DMA LDS writes and the centroid loads visible; the ring stays in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    for (int64_t it = 0; it < my_ntiles; ++it) {
        const int buf = (int)(it % NSTAGE);
        const int64_t tile = (int64_t)blockIdx.x + it * G;
        // prefetch tile it + NSTAGE - 1
        int ahead = 0;
        if (it + NSTAGE - 1 < my_ntiles) {
            stage_tile(lds, (int)((it + NSTAGE - 1) % NSTAGE), X, (tile + (NSTAGE - 1) * G) * TR, N, tid, wave);
            ahead = NSTAGE - 1;
        } else {
            ahead = (int)(my_ntiles - 1 - it);
        }
        wait_vmcnt_n(ahead * GLDS_PER_THREAD);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");

        const char* xb = lds + OFF_X + buf * TILE_BYTES;
        uint32_t* mcur = reinterpret_cast<uint32_t*>(lds + OFF_MASK + (int)(it & 1) * 128 * 16);
        uint32_t* mnext = reinterpret_cast<uint32_t*>(lds + OFF_MASK + (int)((it + 1) & 1) * 128 * 16);
        // clear next parity's masks (last read in iteration it-1, next written in it+1)
        mnext[tid] = 0u;
        mnext[tid + 256] = 0u;

        // ---- 1. distance GEMM: rows 32*wave + l32 ----
        const float* ni = reinterpret_cast<const float*>(lds + OFF_NINIT);
        f32x16 acc[KB];
#pragma unroll
        for (int b = 0; b < KB; ++b) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(ni + 32 * b + 8 * g + 4 * h);
                acc[b][4 * g + 0] = v[0];
                acc[b][4 * g + 1] = v[1];
                acc[b][4 * g + 2] = v[2];
                acc[b][4 * g + 3] = v[3];
            }
        }
        const int myrow = 32 * wave + l32;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xb + xoff(myrow, 2 * s + h));
#pragma unroll
            for (int b = 0; b < KB; ++b)
                acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf[b][s], xv, acc[b], 0, 0, 0);
        }
        // ---- 2. argmax over centroids (index in low 7 mantissa bits) ----
        float best = -3.0e38f;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t c = 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float v = __uint_as_float((__float_as_uint(acc[b][r]) & 0xFFFFFF80u) | c);
                best = fmaxf(best, v);
            }
        }
        best = fmaxf(best, __shfl_xor(best, 32));
        const int64_t grow = tile * TR + myrow;
        if (h == 0 && grow < N) {
            const uint32_t c = __float_as_uint(best) & 127u;
            __hip_atomic_fetch_or(mcur + c * 4 + (myrow >> 5), 1u << (myrow & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        barrier_lds();

        // ---- 3. one-hot accumulate: centroid block = wave ----
        if (wave < KB) {
            const u32x4 mw = *reinterpret_cast<const u32x4*>(mcur + (32 * wave + l32) * 4);
            if (h == 0) cnt += (float)(__popc(mw[0]) + __popc(mw[1]) + __popc(mw[2]) + __popc(mw[3]));
            const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const uint32_t word = mw[s >> 1];
                const uint32_t byte = (word >> (16 * (s & 1) + 8 * h)) & 255u;
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(lds + OFF_LUT + byte * 16);
#pragma unroll
                for (int db = 0; db < 4; ++db) {
                    const int ch = 4 * db + 2 * (g & 1) + (p >> 1);
                    const int r0 = 16 * s + 8 * (g >> 1) + q;
                    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (__attribute__((address_space(3))) bf16x4*)(xb + xoff(r0, ch) + 8 * (p & 1)));
                    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (__attribute__((address_space(3))) bf16x4*)(xb + xoff(r0 + 4, ch) + 8 * (p & 1)));
                    const bf16x8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    sacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, sacc[db], 0, 0, 0);
                }
            }
        }
        barrier_lds();
    }

    // ---- epilogue: partial sums (fp32) of centroid block `wave` ----
    if (wave < KB) {
        float* S = slab + (int64_t)blockIdx.x * 128 * D;
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int c = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
                S[c * D + 32 * db + l32] = sacc[db][r];
            }
        if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wave + l32] = cnt;
    } else {
        float* S = slab + (int64_t)blockIdx.x * 128 * D;
        for (int e = lane; e < 32 * D; e += 64) S[(32 * wave) * D + e] = 0.f;
        if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wave + l32] = 0.f;
    }
}

// ---------------------------------------------------------------------------------------------------
// v2: role-split producer/consumer pipeline, 8 waves (2 per SIMD), ONE barrier per tile.
//   waves 0-3 ("D"): distance GEMM + argmax + mask build for tile i (rows 32w..32w+31)
//   waves 4-7 ("A"): one-hot accumulation of tile i-1 (centroid block w-4)
// so each SIMD co-schedules one matrix-heavy distance wave with one accumulation wave, and VALU
// (argmax), LDS reads and MFMA of the two roles overlap.  X ring: 4 x 32 KiB (tile i-1 still read by
// the A-waves while tiles i+1, i+2 land); masks: 3 rotating buffers.
// ---------------------------------------------------------------------------------------------------
constexpr int V2_NBUF = 4;
constexpr int V2_AHEAD = 2;                              // tiles in flight beyond the current one
constexpr int V2_GLDS = TILE_BYTES / (512 * 16);         // 4 per thread per tile
constexpr int V2_OFF_X = 0;
constexpr int V2_OFF_LUT = V2_NBUF * TILE_BYTES;
constexpr int V2_OFF_MASK = V2_OFF_LUT + 256 * 16;       // [3][128][4] u32
constexpr int V2_OFF_NINIT = V2_OFF_MASK + 3 * 128 * 16;
constexpr int V2_LDS_BYTES = V2_OFF_NINIT + 128 * 4;

__device__ __forceinline__ void v2_stage_tile(char* lds, int buf, const char* X, int64_t row0, int64_t N,
                                              int tid, int wave) {
    char* dst_base = lds + V2_OFF_X + buf * TILE_BYTES;
#pragma unroll
    for (int i = 0; i < V2_GLDS; ++i) {
        const int p = i * 8192 + tid * 16;
        const int row = p >> 8;
        const int chp = (p >> 4) & 15;
        const int chl = chp ^ (((row & 3) << 2) | ((row >> 2) & 3));
        int64_t grow = row0 + row;
        grow = grow < N ? grow : (N - 1);
        const char* src = X + grow * ROWB + chl * 16;
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)LDS_PTR(dst_base + i * 8192 + wave * 1024));
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(m0v)
            : "memory");
    }
}

__device__ __forceinline__ void v2_wait(int ahead) {
    if (ahead >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int KB>
__global__ __launch_bounds__(512, 2) void kmeans_assign_accum_v2_kernel(
    const __bf16* __restrict__ Xp, int64_t N, const __bf16* __restrict__ Cp, const float* __restrict__ ninit,
    float* __restrict__ slab, float* __restrict__ slab_cnt, int64_t ntiles) {
    __shared__ __attribute__((aligned(16))) char lds[V2_LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const bool is_d = wave < 4;
    const int wr = wave & 3;                     // row group (D) / centroid block (A)
    const char* X = reinterpret_cast<const char*>(Xp);
    const int64_t G = gridDim.x;
    const int64_t my_ntiles = (ntiles > (int64_t)blockIdx.x) ? (ntiles - 1 - blockIdx.x) / G + 1 : 0;

    for (int s = 0; s < V2_AHEAD; ++s)
        if (s < my_ntiles) v2_stage_tile(lds, s, X, ((int64_t)blockIdx.x + s * G) * TR, N, tid, wave);
    {
        uint32_t* lut = reinterpret_cast<uint32_t*>(lds + V2_OFF_LUT);
        for (int e = tid; e < 256 * 4; e += 512) {
            const int ent = e >> 2, pair = e & 3;
            const uint32_t b0 = (ent >> (2 * pair)) & 1, b1 = (ent >> (2 * pair + 1)) & 1;
            lut[e] = (b0 ? 0x3F80u : 0u) | (b1 ? 0x3F800000u : 0u);
        }
        uint32_t* m = reinterpret_cast<uint32_t*>(lds + V2_OFF_MASK);
        for (int e = tid; e < 3 * 128 * 4; e += 512) m[e] = 0u;
        float* ni = reinterpret_cast<float*>(lds + V2_OFF_NINIT);
        if (tid < 128) ni[tid] = ninit[tid];
    }
    bf16x8 cf[KB][8];
    if (is_d) {
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int s = 0; s < 8; ++s)
                cf[b][s] = *reinterpret_cast<const bf16x8*>(Cp + (32 * b + l32) * D + 16 * s + 8 * h);
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(cf[b][s]));
    }
    // one accumulator set per wave, role-dependent: D-waves re-initialise it per tile (distance scores),
    // A-waves keep it for the whole kernel (per-centroid-block sums) -> no duplicated register budget
    f32x16 acc[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[db][r] = 0.f;
    float cnt = 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // iteration i: D-waves on tile i (if i < my_ntiles), A-waves on tile i-1 (if i >= 1)
    for (int64_t i = 0; i <= my_ntiles; ++i) {
        // X(i) was issued two iterations ago; X(i+1) (if any) may stay in flight
        v2_wait((i + 1 < my_ntiles) ? 1 : 0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // every wave has left iteration i-1, so buffer (i+2)%4 (tile i-2) is free: refill it
        if (i + V2_AHEAD < my_ntiles)
            v2_stage_tile(lds, (int)((i + V2_AHEAD) % V2_NBUF), X,
                          ((int64_t)blockIdx.x + (i + V2_AHEAD) * G) * TR, N, tid, wave);

        if (is_d) {
            if (i < my_ntiles) {
                const char* xb = lds + V2_OFF_X + (int)(i % V2_NBUF) * TILE_BYTES;
                uint32_t* mcur = reinterpret_cast<uint32_t*>(lds + V2_OFF_MASK + (int)(i % 3) * 128 * 16);
                const float* ni = reinterpret_cast<const float*>(lds + V2_OFF_NINIT);
#pragma unroll
                for (int b = 0; b < KB; ++b)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const f32x4 v = *reinterpret_cast<const f32x4*>(ni + 32 * b + 8 * g + 4 * h);
                        acc[b][4 * g + 0] = v[0];
                        acc[b][4 * g + 1] = v[1];
                        acc[b][4 * g + 2] = v[2];
                        acc[b][4 * g + 3] = v[3];
                    }
                const int myrow = 32 * wr + l32;
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xb + xoff(myrow, 2 * s + h));
#pragma unroll
                    for (int b = 0; b < KB; ++b)
                        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf[b][s], xv, acc[b], 0, 0, 0);
                }
                float best = -3.0e38f;
#pragma unroll
                for (int b = 0; b < KB; ++b)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t c = 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
                        best = fmaxf(best, __uint_as_float((__float_as_uint(acc[b][r]) & 0xFFFFFF80u) | c));
                    }
                best = fmaxf(best, __shfl_xor(best, 32));
                const int64_t grow = ((int64_t)blockIdx.x + i * G) * TR + myrow;
                if (h == 0 && grow < N) {
                    const uint32_t c = __float_as_uint(best) & 127u;
                    __hip_atomic_fetch_or(mcur + c * 4 + (myrow >> 5), 1u << (myrow & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        } else {
            // clear masks of tile i-2 (read by the A-waves in iteration i-1) for tile i+1
            uint32_t* mclr = reinterpret_cast<uint32_t*>(lds + V2_OFF_MASK + (int)((i + 1) % 3) * 128 * 16);
            mclr[tid - 256] = 0u;
            mclr[tid] = 0u;  // tid in [256,512): covers words 256..511
            if (i >= 1 && wr < KB) {
                const int64_t j = i - 1;
                const char* xb = lds + V2_OFF_X + (int)(j % V2_NBUF) * TILE_BYTES;
                const uint32_t* mprev =
                    reinterpret_cast<const uint32_t*>(lds + V2_OFF_MASK + (int)(j % 3) * 128 * 16);
                const u32x4 mw = *reinterpret_cast<const u32x4*>(mprev + (32 * wr + l32) * 4);
                if (h == 0) cnt += (float)(__popc(mw[0]) + __popc(mw[1]) + __popc(mw[2]) + __popc(mw[3]));
                // per-lane tr-read bases: rows 8(g>>1)+q (+4 for the upper half) of k-step 0, chunk group db;
                // k-step s adds s*4096 B (16 rows; the swizzle depends on row & 15 only) -> immediate offsets
                const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
                int tb_lo[4], tb_hi[4];
#pragma unroll
                for (int db = 0; db < 4; ++db) {
                    const int ch = 4 * db + 2 * (g & 1) + (p >> 1);
                    tb_lo[db] = (int)(uintptr_t)LDS_PTR(xb) + xoff(8 * (g >> 1) + q, ch) + 8 * (p & 1);
                    tb_hi[db] = (int)(uintptr_t)LDS_PTR(xb) + xoff(8 * (g >> 1) + q + 4, ch) + 8 * (p & 1);
                }
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const uint32_t word = mw[s >> 1];
                    const uint32_t byte = (word >> (16 * (s & 1) + 8 * h)) & 255u;
                    const bf16x8 a = *reinterpret_cast<const bf16x8*>(lds + V2_OFF_LUT + byte * 16);
#pragma unroll
                    for (int db = 0; db < 4; ++db) {
                        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                            (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tb_lo[db] + s * 4096));
                        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                            (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tb_hi[db] + s * 4096));
                        const bf16x8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                        acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc[db], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    float* S = slab + (int64_t)blockIdx.x * 128 * D;
    if (!is_d) {
        if (wr < KB) {
#pragma unroll
            for (int db = 0; db < 4; ++db)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int c = 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h;
                    S[c * D + 32 * db + l32] = acc[db][r];
                }
            if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wr + l32] = cnt;
        } else {
            for (int e = lane; e < 32 * D; e += 64) S[(32 * wr) * D + e] = 0.f;
            if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wr + l32] = 0.f;
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// v3: register-lean 3-stage pipeline for any k <= 128, 8 waves (2 per SIMD), 64-row tiles, one barrier
// per tile.  Iteration i:
//   D-waves (0-3): wave w -> rows 32*(w&1)..+31 of tile i vs centroid blocks {2(w>>1), 2(w>>1)+1}
//                  (64 centroids, 64 VGPRs of fragments); per-row partial argmax -> pbest[i&1][w>>1][row]
//   A-waves (4-7): (a) combine the two partials of tile i-1 -> per-centroid row masks (ds_or_b32)
//                  (b) one-hot MFMA accumulation of tile i-2 for centroid block (w-4)
// LDS: 6 x 16 KiB X ring (3 tiles in flight), 3 mask sets, 2 pbest sets, LUT, -|c|^2/2.
// ---------------------------------------------------------------------------------------------------
constexpr int V3_TR = 64;
constexpr int V3_TILE = V3_TR * ROWB;                      // 16 KiB
constexpr int V3_NBUF = 6;
constexpr int V3_AHEAD = 3;
constexpr int V3_GLDS = V3_TILE / (512 * 16);             // 2 per thread per tile
constexpr int V3_OFF_LUT = V3_NBUF * V3_TILE;
constexpr int V3_OFF_MASK = V3_OFF_LUT + 256 * 16;        // [3][128 c][2 words]
constexpr int V3_OFF_PBEST = V3_OFF_MASK + 3 * 128 * 8;   // [2][2 halves][64 rows] f32
constexpr int V3_OFF_NINIT = V3_OFF_PBEST + 2 * 2 * 64 * 4;
constexpr int V3_OFF_C = V3_OFF_NINIT + 128 * 4;         // [128 c][128 d] bf16, swizzled like X
constexpr int V3_LDS_BYTES = V3_OFF_C + 128 * ROWB;

__device__ __forceinline__ void v3_stage_tile(char* lds, int buf, const char* X, int64_t row0, int64_t N,
                                              int tid, int wave) {
    char* dst_base = lds + buf * V3_TILE;
#pragma unroll
    for (int i = 0; i < V3_GLDS; ++i) {
        const int p = i * 8192 + tid * 16;
        const int row = p >> 8;
        const int chp = (p >> 4) & 15;
        const int chl = chp ^ (((row & 3) << 2) | ((row >> 2) & 3));
        int64_t grow = row0 + row;
        grow = grow < N ? grow : (N - 1);
        const char* src = X + grow * ROWB + chl * 16;
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)LDS_PTR(dst_base + i * 8192 + wave * 1024));
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(m0v)
            : "memory");
    }
}

__device__ __forceinline__ void v3_wait(int pending_after) {
    // pending_after = number of tiles issued after the one we need (0..2), 2 glds each
    if (pending_after >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (pending_after == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int KB>
__global__ __launch_bounds__(512, 2) void kmeans_assign_accum_v3_kernel(
    const __bf16* __restrict__ Xp, int64_t N, const __bf16* __restrict__ Cp, const float* __restrict__ ninit,
    float* __restrict__ slab, float* __restrict__ slab_cnt, int64_t ntiles) {
    __shared__ __attribute__((aligned(16))) char lds[V3_LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const bool is_d = wave < 4;
    const int wr = wave & 3;
    const char* X = reinterpret_cast<const char*>(Xp);
    const int64_t G = gridDim.x;
    const int64_t my_ntiles = (ntiles > (int64_t)blockIdx.x) ? (ntiles - 1 - blockIdx.x) / G + 1 : 0;

    for (int s = 0; s < V3_AHEAD; ++s)
        if (s < my_ntiles) v3_stage_tile(lds, s, X, ((int64_t)blockIdx.x + s * G) * V3_TR, N, tid, wave);
    {
        uint32_t* lut = reinterpret_cast<uint32_t*>(lds + V3_OFF_LUT);
        for (int e = tid; e < 256 * 4; e += 512) {
            const int ent = e >> 2, pair = e & 3;
            const uint32_t b0 = (ent >> (2 * pair)) & 1, b1 = (ent >> (2 * pair + 1)) & 1;
            lut[e] = (b0 ? 0x3F80u : 0u) | (b1 ? 0x3F800000u : 0u);
        }
        uint32_t* m = reinterpret_cast<uint32_t*>(lds + V3_OFF_MASK);
        for (int e = tid; e < 3 * 128 * 2; e += 512) m[e] = 0u;
        float* ni = reinterpret_cast<float*>(lds + V3_OFF_NINIT);
        if (tid < 128) ni[tid] = ninit[tid];
    }
    // centroids -> LDS (swizzled [c][d] image read by the D-waves as MFMA A operand)
    {
        bf16x8 cv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = r * 512 + tid;  // 16-byte chunk index: row e>>4, chunk e&15
            cv[r] = *reinterpret_cast<const bf16x8*>(Cp + (e >> 4) * D + (e & 15) * 8);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = r * 512 + tid;
            *reinterpret_cast<bf16x8*>(lds + V3_OFF_C + xoff(e >> 4, e & 15)) = cv[r];
        }
    }
    const int cb0 = 2 * (wr >> 1);
    f32x16 acc[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[db][r] = 0.f;
    float cnt = 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    for (int64_t i = 0; i < my_ntiles + 2; ++i) {
        {
            int64_t after = my_ntiles - 1 - i;  // tiles issued after tile i (at most AHEAD-1 = 2 outstanding)
            after = after < 0 ? 0 : (after > 2 ? 2 : after);
            v3_wait((int)after);
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (i + V3_AHEAD < my_ntiles)
            v3_stage_tile(lds, (int)((i + V3_AHEAD) % V3_NBUF), X,
                          ((int64_t)blockIdx.x + (i + V3_AHEAD) * G) * V3_TR, N, tid, wave);

        if (is_d) {
            if (i < my_ntiles && cb0 < KB) {
                const char* xb = lds + (int)(i % V3_NBUF) * V3_TILE;
                const float* ni = reinterpret_cast<const float*>(lds + V3_OFF_NINIT);
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const f32x4 v = *reinterpret_cast<const f32x4*>(ni + 32 * (cb0 + j) + 8 * g + 4 * h);
                        acc[j][4 * g + 0] = v[0];
                        acc[j][4 * g + 1] = v[1];
                        acc[j][4 * g + 2] = v[2];
                        acc[j][4 * g + 3] = v[3];
                    }
                const int myrow = 32 * (wr & 1) + l32;
                const char* cbase = lds + V3_OFF_C;
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xb + xoff(myrow, 2 * s + h));
                    const bf16x8 c0 = *reinterpret_cast<const bf16x8*>(cbase + xoff(32 * cb0 + l32, 2 * s + h));
                    acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c0, xv, acc[0], 0, 0, 0);
                    if (cb0 + 1 < KB) {
                        const bf16x8 c1 =
                            *reinterpret_cast<const bf16x8*>(cbase + xoff(32 * (cb0 + 1) + l32, 2 * s + h));
                        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, xv, acc[1], 0, 0, 0);
                    }
                }
                float best = -3.0e38f;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (cb0 + j < KB) {
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const uint32_t c = 32 * (cb0 + j) + (r & 3) + 8 * (r >> 2) + 4 * h;
                            best = fmaxf(best, __uint_as_float((__float_as_uint(acc[j][r]) & 0xFFFFFF80u) | c));
                        }
                    }
                }
                best = fmaxf(best, __shfl_xor(best, 32));
                if (h == 0) {
                    float* pb = reinterpret_cast<float*>(lds + V3_OFF_PBEST) + (int)(i & 1) * 128 + (wr >> 1) * 64;
                    pb[myrow] = best;
                }
            } else if (i < my_ntiles && h == 0) {
                float* pb = reinterpret_cast<float*>(lds + V3_OFF_PBEST) + (int)(i & 1) * 128 + (wr >> 1) * 64;
                pb[32 * (wr & 1) + l32] = -3.0e38f;
            }
        } else {
            // clear the mask set of tile i-3 (consumed in iteration i-1, rebuilt in iteration i+1)
            {
                uint32_t* mclr = reinterpret_cast<uint32_t*>(lds + V3_OFF_MASK + (int)(i % 3) * 128 * 8);
                mclr[tid - 256] = 0u;
            }
            // (a) combine partials of tile i-1 into its masks
            if (i >= 1 && i <= my_ntiles && wr == 0) {
                const int64_t t = i - 1;
                const float* pb = reinterpret_cast<const float*>(lds + V3_OFF_PBEST) + (int)(t & 1) * 128;
                const float best = fmaxf(pb[lane], pb[64 + lane]);
                const int64_t grow = ((int64_t)blockIdx.x + t * G) * V3_TR + lane;
                if (grow < N) {
                    const uint32_t c = __float_as_uint(best) & 127u;
                    uint32_t* mt = reinterpret_cast<uint32_t*>(lds + V3_OFF_MASK + (int)(t % 3) * 128 * 8);
                    __hip_atomic_fetch_or(mt + c * 2 + (lane >> 5), 1u << (lane & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            // (b) accumulate tile i-2
            if (i >= 2 && wr < KB) {
                const int64_t t = i - 2;
                const char* xb = lds + (int)(t % V3_NBUF) * V3_TILE;
                const uint32_t* mprev = reinterpret_cast<const uint32_t*>(lds + V3_OFF_MASK + (int)(t % 3) * 128 * 8);
                const uint32_t mw0 = mprev[(32 * wr + l32) * 2 + 0];
                const uint32_t mw1 = mprev[(32 * wr + l32) * 2 + 1];
                if (h == 0) cnt += (float)(__popc(mw0) + __popc(mw1));
                const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
                int tb_lo[4], tb_hi[4];
#pragma unroll
                for (int db = 0; db < 4; ++db) {
                    const int ch = 4 * db + 2 * (g & 1) + (p >> 1);
                    tb_lo[db] = (int)(uintptr_t)LDS_PTR(xb) + xoff(8 * (g >> 1) + q, ch) + 8 * (p & 1);
                    tb_hi[db] = (int)(uintptr_t)LDS_PTR(xb) + xoff(8 * (g >> 1) + q + 4, ch) + 8 * (p & 1);
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const uint32_t word = (s >> 1) ? mw1 : mw0;
                    const uint32_t byte = (word >> (16 * (s & 1) + 8 * h)) & 255u;
                    const bf16x8 a = *reinterpret_cast<const bf16x8*>(lds + V3_OFF_LUT + byte * 16);
#pragma unroll
                    for (int db = 0; db < 4; ++db) {
                        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                            (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tb_lo[db] + s * 4096));
                        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                            (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tb_hi[db] + s * 4096));
                        const bf16x8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                        acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc[db], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    float* S = slab + (int64_t)blockIdx.x * 128 * D;
    if (!is_d) {
        if (wr < KB) {
#pragma unroll
            for (int db = 0; db < 4; ++db)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int c = 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h;
                    S[c * D + 32 * db + l32] = acc[db][r];
                }
            if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wr + l32] = cnt;
        } else {
            for (int e = lane; e < 32 * D; e += 64) S[(32 * wr) * D + e] = 0.f;
            if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wr + l32] = 0.f;
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// v4: VALU-lean, one wave per SIMD (4 waves, up to 512 registers each), 128-row tiles, one barrier per
// tile, software-pipelined so the argmax VALU work of tile i is issued between the one-hot MFMAs of
// tile i-1 (profiling v1 showed 12 VALU per MFMA and VALU issue, not MFMA or HBM, bounding it):
//   * LDS-DMA through a per-tile buffer descriptor (buffer_load ... lds): no per-lane 64-bit address math,
//     out-of-range rows read as zero by the hardware bounds check (no clamping);
//   * the -|c|^2/2 init lives in registers and is the C operand of the first distance MFMA (no moves);
//   * all LDS addresses are loop-invariant VGPRs + a per-tile scalar offset;
//   * each wave clears the mask words it consumed, so the mask ring needs no extra phase.
// ---------------------------------------------------------------------------------------------------
constexpr int V4_NBUF = 4;
constexpr int V4_OFF_LUT = V4_NBUF * TILE_BYTES;          // 128 KiB of X ring
constexpr int V4_OFF_MASK = V4_OFF_LUT + 256 * 16;        // [2][128 c][4 words]
constexpr int V4_LDS_BYTES = V4_OFF_MASK + 2 * 128 * 16;

__device__ __forceinline__ void v4_stage(char* lds, int buf, const char* X, int64_t row0, int64_t N,
                                         const uint32_t (&voff)[8], int wave) {
    const int64_t rem = (N - row0) * ROWB;
    const int nbytes = rem < TILE_BYTES ? (int)rem : TILE_BYTES;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(X + row0 * ROWB), (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)LDS_PTR(lds + buf * TILE_BYTES + i * 4096 + wave * 1024));
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

template <int KB, bool DIST, bool ACC>
__device__ __forceinline__ void v4_body(char* lds, int cur_off, int prev_off, uint32_t* mcur, uint32_t* mprev,
                                        const bf16x8 (&cf)[KB][8], const bf16x8 (&cn)[KB], const bf16x8& ones,
                                        const int (&xr)[8],
                                        const int (&tbl)[4], const int (&tbh)[4], f32x16 (&sacc)[4], float& cnt,
                                        int wave, int h, int l32, int lane, int64_t grow) {
    f32x16 acc[KB];
    if constexpr (DIST) {
        // k-step "-1": the accumulator starts at -|c|^2/2 = hi + mid + lo (three bf16 parts) x ones
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const f32x16 z = {};
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cn[b], ones, z, 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const bf16x8 xv = *reinterpret_cast<const bf16x8*>(lds + cur_off + xr[s]);
#pragma unroll
            for (int b = 0; b < KB; ++b)
                acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf[b][s], xv, acc[b], 0, 0, 0);
        }
    }
    float best = -3.0e38f;
    if constexpr (ACC) {
        int tl[4], th[4];
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            tl[db] = tbl[db] + prev_off;
            th[db] = tbh[db] + prev_off;
        }
        const u32x4 mw = *reinterpret_cast<const u32x4*>(mprev + (32 * wave + l32) * 4);
        if (h == 0) {
            cnt += (float)(__popc(mw[0]) + __popc(mw[1]) + __popc(mw[2]) + __popc(mw[3]));
            *reinterpret_cast<u32x4*>(mprev + (32 * wave + l32) * 4) = u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const uint32_t byte = (mw[s >> 1] >> (16 * (s & 1) + 8 * h)) & 255u;
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(lds + V4_OFF_LUT + byte * 16);
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                    (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tl[db] + s * 4096));
                const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                    (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(th[db] + s * 4096));
                const bf16x8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                sacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, sacc[db], 0, 0, 0);
            }
            if constexpr (DIST) {
                // argmax slice of the current tile, interleaved with the one-hot MFMAs of the previous one
                constexpr int PER = (KB * 16 + 7) / 8;
#pragma unroll
                for (int t = 0; t < PER; ++t) {
                    const int v = s * PER + t;
                    if (v < KB * 16) {
                        const int b = v >> 4, r = v & 15;
                        const uint32_t c = 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
                        best = fmaxf(best, __uint_as_float((__float_as_uint(acc[b][r]) & 0xFFFFFF80u) | c));
                    }
                }
            }
        }
    } else if constexpr (DIST) {
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t c = 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
                best = fmaxf(best, __uint_as_float((__float_as_uint(acc[b][r]) & 0xFFFFFF80u) | c));
            }
    }
    if constexpr (DIST) {
        best = fmaxf(best, __shfl_xor(best, 32));
        if (h == 0 && grow >= 0) {
            const uint32_t c = __float_as_uint(best) & 127u;
            const int myrow = 32 * wave + l32;
            __hip_atomic_fetch_or(mcur + c * 4 + (myrow >> 5), 1u << (myrow & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

template <int KB>
__global__ __launch_bounds__(256, 1) void kmeans_assign_accum_v4_kernel(
    const __bf16* __restrict__ Xp, int64_t N, const __bf16* __restrict__ Cp, const float* __restrict__ ninit,
    float* __restrict__ slab, float* __restrict__ slab_cnt, int64_t ntiles, int64_t per) {
    __shared__ __attribute__((aligned(16))) char lds[V4_LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const char* X = reinterpret_cast<const char*>(Xp);
    const int64_t G = gridDim.x;
    // tile schedule: per > 0 -> contiguous run of `per` tiles per workgroup (sequential pages/TLB reach),
    //                per == 0 -> tiles strided by the grid
    const int64_t tbase = per > 0 ? (int64_t)blockIdx.x * per : (int64_t)blockIdx.x;
    const int64_t tstride = per > 0 ? 1 : G;
    const int64_t my_ntiles = per > 0 ? (ntiles > tbase ? (ntiles - tbase < per ? ntiles - tbase : per) : 0)
                                      : ((ntiles > (int64_t)blockIdx.x) ? (ntiles - 1 - blockIdx.x) / G + 1 : 0);

    uint32_t voff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int p = i * 4096 + tid * 16;
        const int row = p >> 8;
        const int chp = (p >> 4) & 15;
        voff[i] = (uint32_t)(row * ROWB + 16 * (chp ^ (((row & 3) << 2) | ((row >> 2) & 3))));
    }
    for (int s = 0; s < 2; ++s)
        if (s < my_ntiles) v4_stage(lds, s, X, (tbase + (int64_t)(s) * tstride) * TR, N, voff, wave);
    {
        uint32_t* lut = reinterpret_cast<uint32_t*>(lds + V4_OFF_LUT);
        for (int e = tid; e < 256 * 4; e += 256) {
            const int ent = e >> 2, pair = e & 3;
            const uint32_t b0 = (ent >> (2 * pair)) & 1, b1 = (ent >> (2 * pair + 1)) & 1;
            lut[e] = (b0 ? 0x3F80u : 0u) | (b1 ? 0x3F800000u : 0u);
        }
        uint32_t* m = reinterpret_cast<uint32_t*>(lds + V4_OFF_MASK);
        for (int e = tid; e < 2 * 128 * 4; e += 256) m[e] = 0u;
    }
    bf16x8 cf[KB][8];
    bf16x8 cn[KB];
    // A operand of the norm k-step: row c = 32b + l32, k = 8h + j: three bf16 parts of -|c|^2/2 (h == 0)
#pragma unroll
    for (int b = 0; b < KB; ++b) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
            cf[b][s] = *reinterpret_cast<const bf16x8*>(Cp + (32 * b + l32) * D + 16 * s + 8 * h);
        const float v = ninit[32 * b + l32];
        const __bf16 p0 = (__bf16)v;
        const float r1 = v - (float)p0;
        const __bf16 p1 = (__bf16)r1;
        const __bf16 p2 = (__bf16)(r1 - (float)p1);
        const __bf16 zb = (__bf16)0.0f;
        cn[b] = (h == 0) ? bf16x8{p0, p1, p2, zb, zb, zb, zb, zb} : bf16x8{zb, zb, zb, zb, zb, zb, zb, zb};
    }
    const __bf16 one = (__bf16)1.0f, zb = (__bf16)0.0f;
    const bf16x8 ones = (h == 0) ? bf16x8{one, one, one, zb, zb, zb, zb, zb} : bf16x8{zb, zb, zb, zb, zb, zb, zb, zb};
#pragma unroll
    for (int b = 0; b < KB; ++b) {
#pragma unroll
        for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(cf[b][s]));
        asm volatile("" ::"v"(cn[b]));
    }
    int xr[8];
    const int myrow = 32 * wave + l32;
#pragma unroll
    for (int s = 0; s < 8; ++s) xr[s] = (int)(uintptr_t)LDS_PTR(lds) + xoff(myrow, 2 * s + h) -
                                        (int)(uintptr_t)LDS_PTR(lds);
    int tbl[4], tbh[4];
    {
        const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            const int ch = 4 * db + 2 * (g & 1) + (p >> 1);
            tbl[db] = (int)(uintptr_t)LDS_PTR(lds) + xoff(8 * (g >> 1) + q, ch) + 8 * (p & 1);
            tbh[db] = (int)(uintptr_t)LDS_PTR(lds) + xoff(8 * (g >> 1) + q + 4, ch) + 8 * (p & 1);
        }
    }
    f32x16 sacc[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[db][r] = 0.f;
    float cnt = 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    uint32_t* mbase = reinterpret_cast<uint32_t*>(lds + V4_OFF_MASK);
    // iteration i: distance/argmax of tile i and one-hot accumulation of tile i-1.  The first and the last
    // iteration are peeled so the steady-state loop is one straight-line body (no phi copies of the
    // persistent accumulators between VGPRs and AGPRs).
    auto iter = [&](int64_t i, auto dist_tag, auto acc_tag) {
        constexpr bool DIST = decltype(dist_tag)::value;
        constexpr bool ACC = decltype(acc_tag)::value;
        if (DIST) {
            if (i + 1 < my_ntiles) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (i + 2 < my_ntiles)
            v4_stage(lds, (int)((i + 2) % V4_NBUF), X, (tbase + (int64_t)((i + 2)) * tstride) * TR, N, voff, wave);
        const int cur_off = (int)(i % V4_NBUF) * TILE_BYTES;
        const int prev_off = (int)((i + V4_NBUF - 1) % V4_NBUF) * TILE_BYTES;
        uint32_t* mcur = mbase + (int)(i & 1) * 128 * 4;
        uint32_t* mprev = mbase + (int)((i + 1) & 1) * 128 * 4;
        const int64_t grow = (tbase + (int64_t)(i) * tstride) * TR + myrow;
        const int64_t gr = (grow < N) ? grow : -1;
        v4_body<KB, DIST, ACC>(lds, cur_off, prev_off, mcur, mprev, cf, cn, ones, xr, tbl, tbh, sacc, cnt, wave,
                               h, l32, lane, gr);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (my_ntiles > 0) {
        iter(0, T_{}, F_{});
        for (int64_t i = 1; i < my_ntiles; ++i) iter(i, T_{}, T_{});
        iter(my_ntiles, F_{}, T_{});
    }

    float* S = slab + (int64_t)blockIdx.x * 128 * D;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int c = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
            S[c * D + 32 * db + l32] = sacc[db][r];
        }
    if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wave + l32] = cnt;
}

// ---------------------------------------------------------------------------------------------------
// v5: block-owning waves.  Wave w owns centroid block w for BOTH GEMMs (32 centroids: 32 VGPRs of
// fragments instead of 128), so registers stay well under 256 and out of the AGPR shuffle that bounded v4
// at k > 64.  64-row tiles, 6-deep LDS ring (3 tiles in flight), one barrier per tile, 3-stage skew:
//   iteration i:  distance(tile i, block w) -> per-block row partial argmax pbest[i&1][w][row]
//                 combine(tile i-1): rows 16w..16w+15 take the max over the 4 block partials -> row masks
//                 accumulate(tile i-2, block w) with the one-hot LUT + ds_read_b64_tr_b16 B fragments
// ---------------------------------------------------------------------------------------------------
constexpr int V5_TR = 64;
constexpr int V5_TILE = V5_TR * ROWB;                      // 16 KiB
constexpr uint32_t V5_NBUF = 8;
constexpr int V5_AHEAD = 4;
constexpr int V5_OFF_LUT = V5_NBUF * V5_TILE;             // 128 KiB ring (4 tiles = 64 KiB in flight)
constexpr int V5_OFF_MASK = V5_OFF_LUT + 256 * 16;        // [3][128 c][2 words]
constexpr int V5_OFF_PBEST = V5_OFF_MASK + 3 * 128 * 8;   // [2][4 blocks][64 rows] f32
constexpr int V5_LDS_BYTES = V5_OFF_PBEST + 2 * 4 * 64 * 4;

__device__ __forceinline__ void v5_stage(char* lds, int buf, const char* X, int64_t row0, int64_t N,
                                         const uint32_t (&voff)[4], int wave) {
    const int64_t rem = (N - row0) * ROWB;
    const int nbytes = rem < V5_TILE ? (int)rem : V5_TILE;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(X + row0 * ROWB), (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)LDS_PTR(lds + buf * V5_TILE + i * 4096 + wave * 1024));
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

template <int KB>
__global__ __launch_bounds__(256, 1) void kmeans_assign_accum_v5_kernel(
    const __bf16* __restrict__ Xp, int64_t N, const __bf16* __restrict__ Cp, const float* __restrict__ ninit,
    float* __restrict__ slab, float* __restrict__ slab_cnt, int64_t ntiles, int64_t per) {
    __shared__ __attribute__((aligned(16))) char lds[V5_LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const char* X = reinterpret_cast<const char*>(Xp);
    const int64_t G = gridDim.x;
    // tile schedule: per > 0 -> contiguous run of `per` tiles per workgroup (sequential pages/TLB reach),
    //                per == 0 -> tiles strided by the grid
    const int64_t tbase = per > 0 ? (int64_t)blockIdx.x * per : (int64_t)blockIdx.x;
    const int64_t tstride = per > 0 ? 1 : G;
    const int64_t my_ntiles = per > 0 ? (ntiles > tbase ? (ntiles - tbase < per ? ntiles - tbase : per) : 0)
                                      : ((ntiles > (int64_t)blockIdx.x) ? (ntiles - 1 - blockIdx.x) / G + 1 : 0);
    const bool active = wave < KB;

    uint32_t voff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = i * 4096 + tid * 16;
        const int row = p >> 8;
        const int chp = (p >> 4) & 15;
        voff[i] = (uint32_t)(row * ROWB + 16 * (chp ^ (((row & 3) << 2) | ((row >> 2) & 3))));
    }
    {
        uint4* ring = reinterpret_cast<uint4*>(lds);
        for (int e = tid; e < V5_NBUF * V5_TILE / 16; e += 256) ring[e] = uint4{0u, 0u, 0u, 0u};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    for (int s = 0; s < V5_AHEAD; ++s)
        if (s < my_ntiles) v5_stage(lds, s, X, (tbase + (int64_t)(s) * tstride) * V5_TR, N, voff, wave);
    {
        uint32_t* lut = reinterpret_cast<uint32_t*>(lds + V5_OFF_LUT);
        for (int e = tid; e < 256 * 4; e += 256) {
            const int ent = e >> 2, pair = e & 3;
            const uint32_t b0 = (ent >> (2 * pair)) & 1, b1 = (ent >> (2 * pair + 1)) & 1;
            lut[e] = (b0 ? 0x3F80u : 0u) | (b1 ? 0x3F800000u : 0u);
        }
        uint32_t* m = reinterpret_cast<uint32_t*>(lds + V5_OFF_MASK);
        for (int e = tid; e < 3 * 128 * 2; e += 256) m[e] = 0u;
        float* pb = reinterpret_cast<float*>(lds + V5_OFF_PBEST);
        for (int e = tid; e < 2 * 4 * 64; e += 256) pb[e] = -3.0e38f;
    }
    // own centroid block: fragments + the norm k-step operand (-|c|^2/2 as three bf16 parts)
    const int cb = wave;
    bf16x8 cf[8];
    bf16x8 cn;
    {
        const __bf16 zb = (__bf16)0.0f;
#pragma unroll
        for (int s = 0; s < 8; ++s)
            cf[s] = active ? *reinterpret_cast<const bf16x8*>(Cp + (32 * cb + l32) * D + 16 * s + 8 * h)
                           : bf16x8{zb, zb, zb, zb, zb, zb, zb, zb};
        const float v = active ? ninit[32 * cb + l32] : -3.0e38f;
        const __bf16 p0 = (__bf16)v;
        const float r1 = v - (float)p0;
        const __bf16 p1 = (__bf16)r1;
        const __bf16 p2 = (__bf16)(r1 - (float)p1);
        cn = (h == 0) ? bf16x8{p0, p1, p2, zb, zb, zb, zb, zb} : bf16x8{zb, zb, zb, zb, zb, zb, zb, zb};
#pragma unroll
        for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(cf[s]));
        asm volatile("" ::"v"(cn));
    }
    const __bf16 one = (__bf16)1.0f, zb = (__bf16)0.0f;
    const bf16x8 ones = (h == 0) ? bf16x8{one, one, one, zb, zb, zb, zb, zb} : bf16x8{zb, zb, zb, zb, zb, zb, zb, zb};
    int xr[2][8];
#pragma unroll
    for (int rg = 0; rg < 2; ++rg)
#pragma unroll
        for (int s = 0; s < 8; ++s) xr[rg][s] = xoff(32 * rg + l32, 2 * s + h);
    int tbl[4], tbh[4];
    {
        const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            const int ch = 4 * db + 2 * (g & 1) + (p >> 1);
            tbl[db] = (int)(uintptr_t)LDS_PTR(lds) + xoff(8 * (g >> 1) + q, ch) + 8 * (p & 1);
            tbh[db] = (int)(uintptr_t)LDS_PTR(lds) + xoff(8 * (g >> 1) + q + 4, ch) + 8 * (p & 1);
        }
    }
    f32x16 sacc[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[db][r] = 0.f;
    float cnt = 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    float* pbest = reinterpret_cast<float*>(lds + V5_OFF_PBEST);
    uint32_t* masks = reinterpret_cast<uint32_t*>(lds + V5_OFF_MASK);

    // Every iteration runs the same straight-line MFMA code (no divergent paths -> no register-file
    // copies at control-flow joins): warm-up/drain iterations operate on zero/stale-but-finite LDS tiles
    // with all-zero row masks, and the combine step (scalar/lane work only) skips tiles that do not exist.
    // 4-stage skew so no step waits on a result produced in the same iteration:
    //   iteration i: distance(tile i) MFMAs, argmax(tile i-1) VALU in their gaps, combine(tile i-2),
    //                one-hot accumulate(tile i-3) with masks/LUT fragments loaded right after the barrier.
    const int nt = (int)my_ntiles;
    const int total = (nt + 3 + 1) & ~1;  // even: the loop body is unrolled twice (acc ping-pong)
    f32x16 accA[2], accB[2];
#pragma unroll
    for (int rg = 0; rg < 2; ++rg)
#pragma unroll
        for (int r = 0; r < 16; ++r) accA[rg][r] = accB[rg][r] = -3.0e38f;

    auto body = [&](const int i, f32x16 (&acc)[2], const f32x16 (&accp)[2]) {
        const uint32_t ui = (uint32_t)i;
        if (i < nt) {
            const int after = nt - 1 - i;  // tiles issued after tile i and still outstanding
            if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (i + V5_AHEAD < nt)
            v5_stage(lds, (int)((ui + V5_AHEAD) % V5_NBUF), X,
                     (tbase + (int64_t)((int64_t)(i + V5_AHEAD)) * tstride) * V5_TR, N, voff, wave);
        // accumulation operands of tile i-3 (masks written by last iteration's combine)
        uint32_t* mp = masks + (int)(ui % 3u) * 256 + (32 * wave + l32) * 2;
        const uint32_t mw0 = mp[0], mw1 = mp[1];
        bf16x8 af[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint32_t word = (s >> 1) ? mw1 : mw0;
            const uint32_t byte = (word >> (16 * (s & 1) + 8 * h)) & 255u;
            af[s] = *reinterpret_cast<const bf16x8*>(lds + V5_OFF_LUT + byte * 16);
        }
        // ---- distance of tile i against the own centroid block; argmax of tile i-1 in the gaps ----
        float best0 = -3.0e38f, best1 = -3.0e38f;
        {
            const int cur = (int)(ui % V5_NBUF) * V5_TILE;
            const f32x16 z = {};
#pragma unroll
            for (int rg = 0; rg < 2; ++rg) acc[rg] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cn, ones, z, 0, 0, 0);
#pragma unroll
            for (int s = 0; s < 8; ++s) {
#pragma unroll
                for (int rg = 0; rg < 2; ++rg) {
                    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(lds + cur + xr[rg][s]);
                    acc[rg] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf[s], xv, acc[rg], 0, 0, 0);
#pragma unroll
                    for (int t2 = 0; t2 < 2; ++t2) {
                        const int r = 2 * s + t2;
                        const uint32_t c = 32 * cb + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const float pk = __uint_as_float((__float_as_uint(accp[rg][r]) & 0xFFFFFF80u) | c);
                        if (rg == 0) best0 = fmaxf(best0, pk);
                        else best1 = fmaxf(best1, pk);
                    }
                }
            }
        }
        best0 = fmaxf(best0, __shfl_xor(best0, 32));
        best1 = fmaxf(best1, __shfl_xor(best1, 32));
        {
            float* pb = pbest + (int)((ui + 1) & 1u) * 256 + wave * 64 + 32 * h;
            pb[l32] = h ? best1 : best0;
        }
        // ---- combine tile i-2 (rows 16w..16w+15): max over the 4 block partials -> row masks ----
        {
            const int t = i - 2;
            const int row = 16 * wave + (lane & 15);
            const int64_t grow = (tbase + (int64_t)((int64_t)t) * tstride) * V5_TR + row;
            if (lane < 16 && t >= 0 && t < nt && grow < N) {
                const float* pb = pbest + (int)(ui & 1u) * 256;
                const float best = fmaxf(fmaxf(pb[row], pb[64 + row]), fmaxf(pb[128 + row], pb[192 + row]));
                const uint32_t c = __float_as_uint(best) & 127u;
                __hip_atomic_fetch_or(masks + (int)((ui + 1) % 3u) * 256 + c * 2 + (row >> 5), 1u << (row & 31),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        // ---- accumulate tile i-3 for the own block ----
        {
            const int po = (int)((ui + V5_NBUF - 3) % V5_NBUF) * V5_TILE;
            cnt += (h == 0) ? (float)(__popc(mw0) + __popc(mw1)) : 0.f;
            mp[h] = 0u;  // both halves read the same pair; lane h clears word h
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
                for (int db = 0; db < 4; ++db) {
                    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tbl[db] + po + s * 4096));
                    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tbh[db] + po + s * 4096));
                    const bf16x8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    sacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bv, sacc[db], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    for (int i = 0; i < total; i += 2) {
        body(i, accA, accB);
        body(i + 1, accB, accA);
    }

    float* S = slab + (int64_t)blockIdx.x * 128 * D;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int c = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
            S[c * D + 32 * db + l32] = sacc[db][r];
        }
    if (h == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * wave + l32] = cnt;
}

// ---------------------------------------------------------------------------------------------------
// v6: v5's block-owning schedule on 8 waves (512 threads, two waves per SIMD) so one wave's LDS/MFMA
// latency stalls are covered by its SIMD partner.  Wave w: centroid block cb = w & 3, half = w >> 2.
//   distance: rows 32*half..+31 of the tile vs block cb (9 MFMAs); combine: rows 8w..8w+7;
//   accumulate: block cb x d-blocks {2*half, 2*half+1} (8 MFMAs).  <= 256 registers per wave.
// Same 64-row tiles / 8-deep ring / 4-stage skew as v5; mask words of tile t are cleared one iteration
// after they are consumed (both halves read them).
// ---------------------------------------------------------------------------------------------------
template <int P0 = 0, int P1 = 2>
__device__ __forceinline__ void v6_stage(char* lds, int buf, const char* X, int64_t row0, int64_t N,
                                         const uint32_t (&voff)[2], int wave) {
    const int64_t rem = (N - row0) * ROWB;
    const int nbytes = rem < V5_TILE ? (int)rem : V5_TILE;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(X + row0 * ROWB), (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int i = P0; i < P1; ++i) {
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)LDS_PTR(lds + buf * V5_TILE + i * 8192 + wave * 1024));
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

#ifndef ALINK_V6_LATE_STAGE
#define ALINK_V6_LATE_STAGE 1
#endif
template <int KB, bool LOAD_ONLY = false, bool COMPUTE_ONLY = false>
__global__ __launch_bounds__(512, 1) void kmeans_assign_accum_v6_kernel(
    const __bf16* __restrict__ Xp, int64_t N, const __bf16* __restrict__ Cp, const float* __restrict__ ninit,
    float* __restrict__ slab, float* __restrict__ slab_cnt, int64_t ntiles, int64_t per) {
    __shared__ __attribute__((aligned(16))) char lds[V5_LDS_BYTES];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cb = wave & 3;
    const int half = wave >> 2;
    const int h = lane >> 5;
    const int l32 = lane & 31;
    const char* X = reinterpret_cast<const char*>(Xp);
    const int64_t G = gridDim.x;
    const int64_t tbase = per > 0 ? (int64_t)blockIdx.x * per : (int64_t)blockIdx.x;
    const int64_t tstride = per > 0 ? 1 : G;
    const int64_t my_ntiles = per > 0 ? (ntiles > tbase ? (ntiles - tbase < per ? ntiles - tbase : per) : 0)
                                      : ((ntiles > (int64_t)blockIdx.x) ? (ntiles - 1 - blockIdx.x) / G + 1 : 0);
    const bool active = cb < KB;

    uint32_t voff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int p = i * 8192 + tid * 16;
        const int row = p >> 8;
        const int chp = (p >> 4) & 15;
        voff[i] = (uint32_t)(row * ROWB + 16 * (chp ^ (((row & 3) << 2) | ((row >> 2) & 3))));
    }
    {
        uint4* ring = reinterpret_cast<uint4*>(lds);
        for (int e = tid; e < (int)(V5_NBUF * V5_TILE / 16); e += 512) ring[e] = uint4{0u, 0u, 0u, 0u};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    }
    for (int s = 0; s < V5_AHEAD; ++s)
        if (s < my_ntiles && !COMPUTE_ONLY) v6_stage(lds, s, X, (tbase + (int64_t)s * tstride) * V5_TR, N, voff, wave);
    {
        uint32_t* lut = reinterpret_cast<uint32_t*>(lds + V5_OFF_LUT);
        for (int e = tid; e < 256 * 4; e += 512) {
            const int ent = e >> 2, pair = e & 3;
            const uint32_t b0 = (ent >> (2 * pair)) & 1, b1 = (ent >> (2 * pair + 1)) & 1;
            lut[e] = (b0 ? 0x3F80u : 0u) | (b1 ? 0x3F800000u : 0u);
        }
        uint32_t* m = reinterpret_cast<uint32_t*>(lds + V5_OFF_MASK);
        for (int e = tid; e < 3 * 128 * 2; e += 512) m[e] = 0u;
        float* pb = reinterpret_cast<float*>(lds + V5_OFF_PBEST);
        for (int e = tid; e < 2 * 4 * 64; e += 512) pb[e] = -3.0e38f;
    }
    bf16x8 cf[8];
    // -|c|^2/2 of the 16 centroids this lane's accumulator registers hold (row r of the 32x32 C block is
    // centroid 32cb + (r&3) + 8(r>>2) + 4h for every sample column): the distance GEMM starts from it as its
    // fp32 C operand, so the norm costs no MFMA k-step and no bf16 splitting
    f32x16 nv;
    const __bf16 zb = (__bf16)0.0f;
    {
#pragma unroll
        for (int s = 0; s < 8; ++s)
            cf[s] = active ? *reinterpret_cast<const bf16x8*>(Cp + (32 * cb + l32) * D + 16 * s + 8 * h)
                           : bf16x8{zb, zb, zb, zb, zb, zb, zb, zb};
#pragma unroll
        for (int r = 0; r < 16; ++r)
            nv[r] = active ? ninit[32 * cb + (r & 3) + 8 * (r >> 2) + 4 * h] : -3.0e38f;
#pragma unroll
        for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(cf[s]));
    }
    int xr[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) xr[s] = xoff(32 * half + l32, 2 * s + h);
    int tbl[2], tbh[2];
    {
        const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int db = 2 * half + j;
            const int ch = 4 * db + 2 * (g & 1) + (p >> 1);
            tbl[j] = (int)(uintptr_t)LDS_PTR(lds) + xoff(8 * (g >> 1) + q, ch) + 8 * (p & 1);
            tbh[j] = (int)(uintptr_t)LDS_PTR(lds) + xoff(8 * (g >> 1) + q + 4, ch) + 8 * (p & 1);
        }
    }
    f32x16 sacc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[j][r] = 0.f;
    float cnt = 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();

    float* pbest = reinterpret_cast<float*>(lds + V5_OFF_PBEST);
    uint32_t* masks = reinterpret_cast<uint32_t*>(lds + V5_OFF_MASK);
    const int nt = (int)my_ntiles;
    const int total = (nt + 3 + 1) & ~1;
    f32x16 accA, accB;
#pragma unroll
    for (int r = 0; r < 16; ++r) accA[r] = accB[r] = -3.0e38f;

    auto body = [&](const int i, f32x16& acc, const f32x16& accp) {
        const uint32_t ui = (uint32_t)i;
        if (i < nt && !COMPUTE_ONLY) {
            const int after = nt - 1 - i;
            if (after >= 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if (after == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if (after == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // ring slot (i+4)%8 held tile i-4, last read by the accumulate of iteration i-1: free anywhere after
        // the barrier.  The LDS-DMA pieces are cheapest to issue outside the MFMA/ds_read phases, so by
        // default they go out in the combine section after the distance GEMM (ALINK_V6_LATE_STAGE).
        const bool stage_now = i + V5_AHEAD < nt && !COMPUTE_ONLY;
        if (!ALINK_V6_LATE_STAGE || LOAD_ONLY) {
            if (stage_now)
                v6_stage(lds, (int)((ui + V5_AHEAD) % V5_NBUF), X,
                         (tbase + (int64_t)(i + V5_AHEAD) * tstride) * V5_TR, N, voff, wave);
        }
        if constexpr (LOAD_ONLY) return;
        // masks of tile i-3 (set i%3); the set consumed last iteration ((i+2)%3) is cleared by half 0
        uint32_t* mp = masks + (int)(ui % 3u) * 256 + (32 * cb + l32) * 2;
        const uint32_t mw0 = mp[0], mw1 = mp[1];
        if (half == 0) masks[(int)((ui + 2) % 3u) * 256 + (32 * cb + l32) * 2 + h] = 0u;
        bf16x8 af[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint32_t word = (s >> 1) ? mw1 : mw0;
            const uint32_t byte = (word >> (16 * (s & 1) + 8 * h)) & 255u;
            af[s] = *reinterpret_cast<const bf16x8*>(lds + V5_OFF_LUT + byte * 16);
        }
        // ---- distance of tile i (own rows, own block); argmax of tile i-1 in the gaps ----
        float best = -3.0e38f;
        {
            const int cur = (int)(ui % V5_NBUF) * V5_TILE;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const bf16x8 xv = *reinterpret_cast<const bf16x8*>(lds + cur + xr[s]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cf[s], xv, s == 0 ? nv : acc, 0, 0, 0);
#pragma unroll
                for (int t2 = 0; t2 < 2; ++t2) {
                    const int r = 2 * s + t2;
                    const uint32_t c = 32 * cb + (r & 3) + 8 * (r >> 2) + 4 * h;
                    best = fmaxf(best, __uint_as_float((__float_as_uint(accp[r]) & 0xFFFFFF80u) | c));
                }
            }
        }
        best = fmaxf(best, __shfl_xor(best, 32));
        if (h == 0) pbest[(int)((ui + 1) & 1u) * 256 + cb * 64 + 32 * half + l32] = best;
        if (ALINK_V6_LATE_STAGE == 1 || ALINK_V6_LATE_STAGE == 3) {
            if (stage_now)
                v6_stage<0, (ALINK_V6_LATE_STAGE == 1 ? 2 : 1)>(lds, (int)((ui + V5_AHEAD) % V5_NBUF), X,
                         (tbase + (int64_t)(i + V5_AHEAD) * tstride) * V5_TR, N, voff, wave);
        }
        // ---- combine tile i-2 (rows 8w..8w+7) ----
        {
            const int t = i - 2;
            const int row = 8 * wave + (lane & 7);
            const int64_t grow = (tbase + (int64_t)t * tstride) * V5_TR + row;
            if (lane < 8 && t >= 0 && t < nt && grow < N) {
                const float* pb = pbest + (int)(ui & 1u) * 256;
                const float bb = fmaxf(fmaxf(pb[row], pb[64 + row]), fmaxf(pb[128 + row], pb[192 + row]));
                const uint32_t c = __float_as_uint(bb) & 127u;
                __hip_atomic_fetch_or(masks + (int)((ui + 1) % 3u) * 256 + c * 2 + (row >> 5), 1u << (row & 31),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        // ---- accumulate tile i-3: block cb x d-blocks 2*half, 2*half+1 ----
        {
            const int po = (int)((ui + V5_NBUF - 3) % V5_NBUF) * V5_TILE;
            cnt += (h == 0 && half == 0) ? (float)(__popc(mw0) + __popc(mw1)) : 0.f;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tbl[j] + po + s * 4096));
                    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
                        (__attribute__((address_space(3))) bf16x4*)(uintptr_t)(tbh[j] + po + s * 4096));
                    const bf16x8 bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bv, sacc[j], 0, 0, 0);
                }
            }
        }
        if (ALINK_V6_LATE_STAGE == 2 || ALINK_V6_LATE_STAGE == 3) {
            if (stage_now)
                v6_stage<(ALINK_V6_LATE_STAGE == 2 ? 0 : 1), 2>(lds, (int)((ui + V5_AHEAD) % V5_NBUF), X,
                         (tbase + (int64_t)(i + V5_AHEAD) * tstride) * V5_TR, N, voff, wave);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    for (int i = 0; i < total; i += 2) {
        body(i, accA, accB);
        body(i + 1, accB, accA);
    }

    float* S = slab + (int64_t)blockIdx.x * 128 * D;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int c = 32 * cb + (r & 3) + 8 * (r >> 2) + 4 * h;
            S[c * D + 32 * (2 * half + j) + l32] = sacc[j][r];
        }
    if (h == 0 && half == 0) slab_cnt[(int64_t)blockIdx.x * 128 + 32 * cb + l32] = cnt;
}

// fixed-order fp64 reduction of the per-workgroup slabs -> out[k][D+1] (last column = count).
// Block (c, y): y < 4 -> dims 32y..32y+31, y == 4 -> the count; 8 lane groups stride the slabs (coalesced
// 128-B rows), then group partials are added in group order, so the result is run-to-run deterministic.
__global__ __launch_bounds__(256) void kmeans_reduce_slabs_kernel(const float* __restrict__ slab,
                                                                  const float* __restrict__ slab_cnt, int nslab,
                                                                  int k, double* __restrict__ out) {
    __shared__ double part[8][32];
    const int c = blockIdx.x, y = blockIdx.y;
    const int d = threadIdx.x & 31, g = threadIdx.x >> 5;
    double s = 0.0;
    if (y < 4) {
        const float* p = slab + (int64_t)c * D + 32 * y + d;
        for (int w = g; w < nslab; w += 8) s += (double)p[(int64_t)w * 128 * D];
    } else if (d == 0) {
        for (int w = g; w < nslab; w += 8) s += (double)slab_cnt[(int64_t)w * 128 + c];
    }
    part[g][d] = s;
    __syncthreads();
    if (g == 0) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j) t += part[j][d];
        if (y < 4) out[(int64_t)c * (D + 1) + 32 * y + d] = t;
        else if (d == 0) out[(int64_t)c * (D + 1) + D] = t;
    }
}

// next-step centroid operands from fp64 centroids C [k][D]: bf16 block [128][D] (zero rows past k) and the
// accumulator init -|bf16(c)|^2/2 (-3e38 past k), one launch instead of a chain of small torch ops.
__global__ __launch_bounds__(128) void kmeans_prep_centroids_kernel(const double* __restrict__ C, int k,
                                                                    __bf16* __restrict__ cpad,
                                                                    float* __restrict__ ninit) {
    __shared__ float red[128];
    const int c = blockIdx.x, d = threadIdx.x;
    const __bf16 b = c < k ? (__bf16)(float)C[(int64_t)c * D + d] : (__bf16)0.0f;
    cpad[c * D + d] = b;
    const float f = (float)b;
    red[d] = f * f;
    __syncthreads();
    for (int off = 64; off > 0; off >>= 1) {
        if (d < off) red[d] += red[d + off];
        __syncthreads();
    }
    if (d == 0) ninit[c] = c < k ? -0.5f * red[0] : -3.0e38f;
}

}  // namespace

extern "C" {

int alink_kmeans_lds_bytes() { return LDS_BYTES; }

// returns 0 on success, hipError_t otherwise
int alink_kmeans_assign_accum_bf16(const void* X, int64_t N, const void* C, const float* ninit, int k,
                                   float* slab, float* slab_cnt, int grid, void* stream) {
    if (N <= 0 || k < 1 || k > 128 || grid <= 0) return -1;
    const int KB = (k + 31) / 32;
    const int64_t ntiles = (N + TR - 1) / TR;
    if (grid > ntiles) grid = (int)ntiles;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (KB) {
        case 1: hipLaunchKernelGGL(kmeans_assign_accum_kernel<1>, dim3(grid), dim3(256), 0, st,
                                   (const __bf16*)X, N, (const __bf16*)C, ninit, slab, slab_cnt, ntiles); break;
        case 2: hipLaunchKernelGGL(kmeans_assign_accum_kernel<2>, dim3(grid), dim3(256), 0, st,
                                   (const __bf16*)X, N, (const __bf16*)C, ninit, slab, slab_cnt, ntiles); break;
        case 3: hipLaunchKernelGGL(kmeans_assign_accum_kernel<3>, dim3(grid), dim3(256), 0, st,
                                   (const __bf16*)X, N, (const __bf16*)C, ninit, slab, slab_cnt, ntiles); break;
        default: hipLaunchKernelGGL(kmeans_assign_accum_kernel<4>, dim3(grid), dim3(256), 0, st,
                                    (const __bf16*)X, N, (const __bf16*)C, ninit, slab, slab_cnt, ntiles); break;
    }
    return (int)hipGetLastError();
}

int alink_kmeans_assign_accum_bf16_v2(const void* X, int64_t N, const void* C, const float* ninit, int k,
                                      float* slab, float* slab_cnt, int grid, void* stream) {
    if (N <= 0 || k < 1 || k > 128 || grid <= 0) return -1;
    const int KB = (k + 31) / 32;
    const int64_t ntiles = (N + TR - 1) / TR;
    if (grid > ntiles) grid = (int)ntiles;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define V2_LAUNCH(KBV)                                                                                   \
    hipLaunchKernelGGL(kmeans_assign_accum_v2_kernel<KBV>, dim3(grid), dim3(512), 0, st, (const __bf16*)X, N, \
                       (const __bf16*)C, ninit, slab, slab_cnt, ntiles)
    switch (KB) {
        case 1: V2_LAUNCH(1); break;
        case 2: V2_LAUNCH(2); break;
        case 3: V2_LAUNCH(3); break;
        default: V2_LAUNCH(4); break;
    }
#undef V2_LAUNCH
    return (int)hipGetLastError();
}

int alink_kmeans_assign_accum_bf16_v3(const void* X, int64_t N, const void* C, const float* ninit, int k,
                                      float* slab, float* slab_cnt, int grid, void* stream) {
    if (N <= 0 || k < 1 || k > 128 || grid <= 0) return -1;
    const int KB = (k + 31) / 32;
    const int64_t ntiles = (N + V3_TR - 1) / V3_TR;
    if (grid > ntiles) grid = (int)ntiles;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define V3_LAUNCH(KBV)                                                                                   \
    hipLaunchKernelGGL(kmeans_assign_accum_v3_kernel<KBV>, dim3(grid), dim3(512), 0, st, (const __bf16*)X, N, \
                       (const __bf16*)C, ninit, slab, slab_cnt, ntiles)
    switch (KB) {
        case 1: V3_LAUNCH(1); break;
        case 2: V3_LAUNCH(2); break;
        case 3: V3_LAUNCH(3); break;
        default: V3_LAUNCH(4); break;
    }
#undef V3_LAUNCH
    return (int)hipGetLastError();
}

int alink_kmeans_assign_accum_bf16_v4(const void* X, int64_t N, const void* C, const float* ninit, int k,
                                      float* slab, float* slab_cnt, int grid, void* stream, int contiguous) {
    if (N <= 0 || k < 1 || k > 128 || grid <= 0) return -1;
    const int KB = (k + 31) / 32;
    const int64_t ntiles = (N + TR - 1) / TR;
    if (grid > ntiles) grid = (int)ntiles;
    const int64_t per = contiguous ? (ntiles + grid - 1) / grid : 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define V4_LAUNCH(KBV)                                                                                   \
    hipLaunchKernelGGL(kmeans_assign_accum_v4_kernel<KBV>, dim3(grid), dim3(256), 0, st, (const __bf16*)X, N, \
                       (const __bf16*)C, ninit, slab, slab_cnt, ntiles, per)
    switch (KB) {
        case 1: V4_LAUNCH(1); break;
        case 2: V4_LAUNCH(2); break;
        case 3: V4_LAUNCH(3); break;
        default: V4_LAUNCH(4); break;
    }
#undef V4_LAUNCH
    return (int)hipGetLastError();
}

int alink_kmeans_assign_accum_bf16_v5(const void* X, int64_t N, const void* C, const float* ninit, int k,
                                      float* slab, float* slab_cnt, int grid, void* stream, int contiguous) {
    if (N <= 0 || k < 1 || k > 128 || grid <= 0) return -1;
    const int KB = (k + 31) / 32;
    const int64_t ntiles = (N + V5_TR - 1) / V5_TR;
    if (grid > ntiles) grid = (int)ntiles;
    const int64_t per = contiguous ? (ntiles + grid - 1) / grid : 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define V5_LAUNCH(KBV)                                                                                   \
    hipLaunchKernelGGL(kmeans_assign_accum_v5_kernel<KBV>, dim3(grid), dim3(256), 0, st, (const __bf16*)X, N, \
                       (const __bf16*)C, ninit, slab, slab_cnt, ntiles, per)
    switch (KB) {
        case 1: V5_LAUNCH(1); break;
        case 2: V5_LAUNCH(2); break;
        case 3: V5_LAUNCH(3); break;
        default: V5_LAUNCH(4); break;
    }
#undef V5_LAUNCH
    return (int)hipGetLastError();
}

int alink_kmeans_assign_accum_bf16_v6(const void* X, int64_t N, const void* C, const float* ninit, int k,
                                      float* slab, float* slab_cnt, int grid, void* stream, int contiguous) {
    if (N <= 0 || k < 1 || k > 128 || grid <= 0) return -1;
    const int KB = (k + 31) / 32;
    const int64_t ntiles = (N + V5_TR - 1) / V5_TR;
    if (grid > ntiles) grid = (int)ntiles;
    const int64_t per = contiguous ? (ntiles + grid - 1) / grid : 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (contiguous == 4) {  // diagnostics: the compute alone (tiles never loaded; results meaningless)
        hipLaunchKernelGGL((kmeans_assign_accum_v6_kernel<4, false, true>), dim3(grid), dim3(512), 0, st,
                           (const __bf16*)X, N, (const __bf16*)C, ninit, slab, slab_cnt, ntiles, per);
        return (int)hipGetLastError();
    }
    if (contiguous >= 2) {  // diagnostics: the load pipeline alone (no compute; slabs not written)
        hipLaunchKernelGGL((kmeans_assign_accum_v6_kernel<4, true>), dim3(grid), dim3(512), 0, st, (const __bf16*)X,
                           N, (const __bf16*)C, ninit, slab, slab_cnt, ntiles, contiguous == 2 ? per : 0);
        return (int)hipGetLastError();
    }
#define V6_LAUNCH(KBV)                                                                                   \
    hipLaunchKernelGGL(kmeans_assign_accum_v6_kernel<KBV>, dim3(grid), dim3(512), 0, st, (const __bf16*)X, N, \
                       (const __bf16*)C, ninit, slab, slab_cnt, ntiles, per)
    switch (KB) {
        case 1: V6_LAUNCH(1); break;
        case 2: V6_LAUNCH(2); break;
        case 3: V6_LAUNCH(3); break;
        default: V6_LAUNCH(4); break;
    }
#undef V6_LAUNCH
    return (int)hipGetLastError();
}

int alink_kmeans_reduce_slabs(const float* slab, const float* slab_cnt, int nslab, int k, double* out,
                              void* stream) {
    if (k < 1 || k > 128 || nslab < 1) return -1;
    hipLaunchKernelGGL(kmeans_reduce_slabs_kernel, dim3(k, 5), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       slab, slab_cnt, nslab, k, out);
    return (int)hipGetLastError();
}

int alink_kmeans_prep_centroids(const double* C, int k, void* cpad, float* ninit, void* stream) {
    if (k < 0 || k > 128) return -1;
    hipLaunchKernelGGL(kmeans_prep_centroids_kernel, dim3(128), dim3(128), 0, reinterpret_cast<hipStream_t>(stream),
                       C, k, (__bf16*)cpad, ninit);
    return (int)hipGetLastError();
}

}  // extern "C"
