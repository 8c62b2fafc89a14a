// Shared device helpers of the KMeans MFMA tile kernels (kmeans_v7.hip, kmeans_accum.hip) — gfx950 / MI355X.
// 64-row x 128-dim bf16 tiles streamed HBM -> LDS with LDS-DMA (buffer_load ... lds), the bank-conflict-free X
// tile swizzle and one-hot image layout (tools/lds_bank_check.py), and the LDS barrier / vmcnt wait helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kmtile {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

constexpr int D = 128;
constexpr int ROWB = D * 2;                // 256 B per row
constexpr int TR = 64;                     // rows per tile
constexpr int TILE = TR * ROWB;            // 16 KiB
constexpr int LDS_CAP = 160 * 1024;

constexpr uint32_t NONE = 0xFFFFu;

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

// VAR >= 1: the 4 accumulate waves issue 4 pieces per tile each
__device__ __forceinline__ void wait_tile4(int younger) {
    if (younger >= 5) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (younger == 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// stage one 64-row tile with NP pieces per wave (NP = 2: all 8 waves; NP = 4: the 4 accumulate waves, `wave` =
// 0..3 among them); rows past N read as zero (buffer bounds).  NT = 1 issues the pieces with the streaming
// (non-temporal) cache policy: X is read once per superstep, so there is nothing to keep in L2
template <int NP, int NT = 0>
__device__ __forceinline__ void stage_np(char* lds, int slot, const char* X, int64_t row0, int64_t N,
                                         const uint32_t (&voff)[4], int wave) {
    const int64_t rem = (N - row0) * ROWB;
    const int nbytes = rem < TILE ? (int)rem : TILE;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(X + row0 * ROWB), (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(LDS_AS void*)(lds + slot * TILE + i * (TILE / NP) + wave * 1024));
        uint32_t keep;
        if constexpr (NT)
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %3\n\t"
                "s_nop 0\n\t"
                "buffer_load_dwordx4 %1, %2, 0 offen nt lds\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(voff[i]), "s"(rs), "s"(m0v)
                : "memory");
        else
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

// s_waitcnt vmcnt(N) for a compile-time N (0..63)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until the tile `younger` tiles before the newest one issued has landed, NP pieces per tile per wave
template <int NP, int MAXY>
__device__ __forceinline__ void wait_tile_np(int younger) {
    if constexpr (MAXY <= 0) {
        wait_vm<0>();
    } else {
        if (younger >= MAXY) wait_vm<NP * MAXY>();
        else wait_tile_np<NP, MAXY - 1>(younger);
    }
}

}  // namespace kmtile
