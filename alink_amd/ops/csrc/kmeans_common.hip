// KMeans helpers shared by the fused assign+accumulate kernel (kmeans_v7.hip) — CDNA4 (gfx950 / MI355X).
//
//   * kmeans_reduce_slabs: fixed-order fp64 reduction of the per-workgroup fp32 partial sums / counts into the
//     [k][D+1] buffer that the BSP AllReduce sums across GPUs (the reference's centroidAllReduce buffer,
//     A/operator/common/clustering/kmeans/KMeansAssignCluster.java:48-63).  Fixed order -> run-to-run
//     deterministic, independent of workgroup scheduling.
//   * kmeans_prep_centroids: next-superstep centroid operands from the fp64 centroids (KMeansUpdateCentroids
//     output): bf16 block [128][D] and the MFMA accumulator init -|c|^2/2, one launch.
//
// Earlier assign+accumulate designs (v1-v6: 128-row tiles with LUT one-hot, block-owning waves, ...) and the v8
// software-pipelined variant are documented with their measurements in profiles/kmeans_variants.txt and
// profiles/kmeans_v7_v8_pmc.txt; only v7 ships.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstring>

namespace {

constexpr int D = 128;

// fixed-order fp64 reduction of the per-workgroup slabs -> out[k][D+1] (last column = count).
// Block (c, y): y < 4 -> dims 32y..32y+31, y == 4 -> the count; 8 lane groups stride the slabs (coalesced
// 128-B rows), then group partials are added in group order, so the result is run-to-run deterministic.
__global__ __launch_bounds__(256) void kmeans_reduce_slabs_kernel(const float* __restrict__ slab,
                                                                  const float* __restrict__ slab_cnt, int nslab,
                                                                  int k, double* __restrict__ out,
                                                                  const unsigned* __restrict__ skip) {
    // a skipped speculative assign launch left the slabs stale: its reduction is dropped by the host too, so it
    // returns at once on the same word (uniform early return, before any barrier)
    if (skip != nullptr && __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    __shared__ double part[8][32];
    const int c = blockIdx.x, y = blockIdx.y;
    const int d = threadIdx.x & 31, g = threadIdx.x >> 5;
    // four independent partial sums per thread (slabs g, g+8, g+16, g+24 mod 32): the loads of a thread are
    // in flight together instead of one dependent chain; the combination order is fixed -> deterministic
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    if (y < 4) {
        const float* p = slab + (int64_t)c * D + 32 * y + d;
        int w = g;
        for (; w + 24 < nslab; w += 32) {
#pragma unroll
            for (int j = 0; j < 4; ++j) s4[j] += (double)p[(int64_t)(w + 8 * j) * 128 * D];
        }
        for (int j = 0; w < nslab; w += 8, ++j) s4[j & 3] += (double)p[(int64_t)w * 128 * D];
    } else if (d == 0) {
        int w = g;
        for (; w + 24 < nslab; w += 32) {
#pragma unroll
            for (int j = 0; j < 4; ++j) s4[j] += (double)slab_cnt[(int64_t)(w + 8 * j) * 128 + c];
        }
        for (int j = 0; w < nslab; w += 8, ++j) s4[j & 3] += (double)slab_cnt[(int64_t)w * 128 + c];
    }
    const double s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
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

// fused centroid update after the all-reduce (reference KMeansUpdateCentroidsAndSetAllReduce + the termination
// test KMeansIterTermination, A/operator/common/clustering/kmeans/): one workgroup per padded centroid row
//   C[c] = sum[c] / cnt[c]                       (fp64, written for c < k)
//   cpad[c] = bf16(C[c]) (or the held operand, hyst), ninit[c] = -|cpad[c]|^2/2   (the NEXT superstep's MFMA
//   operands: no separate prep launch)
//   stat[0] = max_c ||C[c] - prev[c]||  (fp64 bits, atomicMax: non-negative doubles order as unsigned integers)
//   stat[1] = 1 if any cnt[c] <= 0 (the host then redoes the update with empty-cluster compaction)
// replacing ~8 small torch launches + the prep launch of the next step and giving the host ONE 16-byte read.
__global__ __launch_bounds__(128) void kmeans_update_kernel(const double* __restrict__ buf, int k,
                                                            const double* __restrict__ prev,
                                                            double* __restrict__ C, __bf16* __restrict__ cpad,
                                                            float* __restrict__ ninit,
                                                            unsigned long long* __restrict__ stat, int hyst,
                                                            unsigned long long* __restrict__ host_out, double tol,
                                                            unsigned* __restrict__ skip, unsigned long long seq) {
    __shared__ float red[128];
    __shared__ double redd[128];
    const int c = blockIdx.x, d = threadIdx.x;
    double v = 0.0;
    bool empty = false;
    if (c < k) {
        const double cnt = buf[(int64_t)c * (D + 1) + D];
        empty = !(cnt > 0.0);
        v = empty ? 0.0 : buf[(int64_t)c * (D + 1) + d] / cnt;
        C[(int64_t)c * D + d] = v;
    }
    __bf16 b = (__bf16)(float)v;
    if (hyst) {
        // operand hysteresis: keep the current bf16 operand while the fp64 centroid stays within one bf16 ulp
        // of the row's largest coordinate (the resolution the bf16 dot product has anyway).  Re-quantising every
        // step lets boundary rows flip on sub-ulp centroid jitter, which keeps Lloyd cycling at a ~2e-3 shift
        // floor above epsilon; with the operands held, the assignments (and hence the fp64 centroids) become
        // exactly stationary and the shift reaches 0.
        red[d] = (float)fabs(v);
        __syncthreads();
        for (int off = 64; off > 0; off >>= 1) {
            if (d < off) red[d] = fmaxf(red[d], red[d + off]);
            __syncthreads();
        }
        const float m = red[0];
        __syncthreads();
        if (c < k && m > 0.0f) {
            const float ob = (float)cpad[c * D + d];
            if (fabs(v - (double)ob) < (double)ldexpf(1.0f, ilogbf(m) - 7)) b = (__bf16)ob;
        }
    }
    cpad[c * D + d] = b;
    const float f = (float)b;
    red[d] = f * f;
    const double df = (c < k && prev != nullptr) ? v - prev[(int64_t)c * D + d] : 0.0;
    redd[d] = df * df;
    __syncthreads();
    for (int off = 64; off > 0; off >>= 1) {
        if (d < off) {
            red[d] += red[d + off];
            redd[d] += redd[d + off];
        }
        __syncthreads();
    }
    if (d == 0) {
        ninit[c] = c < k ? -0.5f * red[0] : -3.0e38f;
        if (c < k) {
            const double sh = sqrt(redd[0]);
            atomicMax(stat, (unsigned long long)__double_as_longlong(sh));
            if (empty) atomicMax(stat + 1, 1ull);
        }
        if (host_out != nullptr) {
            // last block to finish publishes the two stats straight into mapped host memory and re-arms the
            // device words (stat[2] = ticket) for the next launch: no memset before and no copy after the kernel
            __threadfence();
            const unsigned long long t = atomicAdd(stat + 2, 1ull);
            if (t == (unsigned long long)gridDim.x - 1) {
                __threadfence();
                const unsigned long long s0 = atomicAdd(stat, 0ull), s1 = atomicAdd(stat + 1, 0ull);
                __hip_atomic_store(host_out, s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(host_out + 1, s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (seq != 0ull) {
                    // launch sequence number after the stats: a host polling host_out[2] == seq reads host_out[0..1]
                    // without an event between this kernel and the work queued after it
                    __threadfence_system();
                    __hip_atomic_store(host_out + 2, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                if (skip != nullptr) {
                    // the next superstep will not run on these centroids: an empty cluster (the host compacts and
                    // relaunches) or converged by the host's own test (max shift < tol on the same double) — a
                    // speculative next-superstep assign launched with this word returns at once
                    const unsigned drop =
                        s1 != 0ull || (prev != nullptr && __longlong_as_double((long long)s0) < tol);
                    __hip_atomic_store(skip, drop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __threadfence_system();
                atomicExch(stat, 0ull);
                atomicExch(stat + 1, 0ull);
                atomicExch(stat + 2, 0ull);
            }
        }
    }
}

}  // namespace

extern "C" {

// buf [k][D+1] (sums | count), prev [k][D] (nullable), C out [k][D], cpad [128][D] bf16, ninit [128],
// stat [3] u64 device words: max shift (double bits), any-empty flag, completion ticket.
// host_out == nullptr: stat[0..1] are zeroed here (memset) and hold the result after the kernel.
// host_out != nullptr (device address of mapped host memory, alink_kmeans_host_stat_alloc): stat must be all-zero
// before the FIRST launch; the kernel's last block writes host_out[0..1] and re-zeroes stat itself.
// hyst != 0: bf16 operand hysteresis (keep cpad[c][d] while |C[c][d] - cpad[c][d]| < one bf16 ulp of max_d |C[c][d]|;
// cpad should hold the operands of the step just run, but any contents are safe: a kept value is that close to C)
// skip != nullptr (needs host_out): the last block also writes *skip = 1 when some cluster is empty or (prev given)
// the max shift is < tol (the termination test), else 0 — read by a speculative next-superstep assign launch
// seq != 0 (needs host_out): host_out[2] = seq is written after the two stats (host completion poll)
int alink_kmeans_update2(const double* buf, int k, const double* prev, double* C, void* cpad, float* ninit,
                         unsigned long long* stat, int hyst, unsigned long long* host_out, double tol, unsigned* skip,
                         unsigned long long seq, void* stream) {
    if (k < 1 || k > 128 || ((skip != nullptr || seq != 0ull) && host_out == nullptr)) return -1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (host_out == nullptr && hipMemsetAsync(stat, 0, 2 * sizeof(unsigned long long), st) != hipSuccess) return -2;
    hipLaunchKernelGGL(kmeans_update_kernel, dim3(128), dim3(128), 0, st, buf, k, prev, C, (__bf16*)cpad, ninit,
                       stat, hyst, host_out, tol, skip, seq);
    return (int)hipGetLastError();
}

int alink_kmeans_update(const double* buf, int k, const double* prev, double* C, void* cpad, float* ninit,
                        unsigned long long* stat, int hyst, unsigned long long* host_out, void* stream) {
    return alink_kmeans_update2(buf, k, prev, C, cpad, ninit, stat, hyst, host_out, 0.0, nullptr, 0ull, stream);
}

// 32 bytes of mapped, coherent pinned host memory for the update's stats: *host = host address, *dev = the
// address kernels write through.
int alink_kmeans_host_stat_alloc(void** host, void** dev) {
    hipError_t e = hipHostMalloc(host, 32, hipHostMallocMapped);
    if (e != hipSuccess) return (int)e;
    memset(*host, 0, 32);
    return (int)hipHostGetDevicePointer(dev, *host, 0);
}

int alink_kmeans_host_stat_free(void* host) { return (int)hipHostFree(host); }

// skip (nullable): the update's skip word; when nonzero at run time the reduction returns at once (out untouched)
int alink_kmeans_reduce_slabs2(const float* slab, const float* slab_cnt, int nslab, int k, double* out,
                               const void* skip, void* stream) {
    if (k < 1 || k > 128 || nslab < 1) return -1;
    hipLaunchKernelGGL(kmeans_reduce_slabs_kernel, dim3(k, 5), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       slab, slab_cnt, nslab, k, out, (const unsigned*)skip);
    return (int)hipGetLastError();
}

int alink_kmeans_reduce_slabs(const float* slab, const float* slab_cnt, int nslab, int k, double* out,
                              void* stream) {
    return alink_kmeans_reduce_slabs2(slab, slab_cnt, nslab, k, out, nullptr, stream);
}

int alink_kmeans_prep_centroids(const double* C, int k, void* cpad, float* ninit, void* stream) {
    if (k < 0 || k > 128) return -1;
    hipLaunchKernelGGL(kmeans_prep_centroids_kernel, dim3(128), dim3(128), 0, reinterpret_cast<hipStream_t>(stream),
                       C, k, (__bf16*)cpad, ninit);
    return (int)hipGetLastError();
}

}  // extern "C"
