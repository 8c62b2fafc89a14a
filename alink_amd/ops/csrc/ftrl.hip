// Hogwild FTRL-proximal on CDNA4 (gfx950 / MI355X) for high-throughput online logistic regression.
//
// Same per-coordinate rule as the reference's CalcTask (FtrlTrainStreamOp.java:396-485) and the sequential host
// loop (_native/csrc/ftrl.cpp):
//   g = (p - y) x_i;  sigma = (sqrt(n_i + g^2) - sqrt(n_i)) / alpha;  z_i += g - sigma w_i;  n_i += g^2
//   w_i = |z_i| <= l1 ? 0 : (sign(z_i) l1 - z_i) / (beta + sqrt(n_i)/alpha + l2)
// but the samples of a micro-batch are processed CONCURRENTLY, one 64-wide wave per sample (grid-strided):
// the wave's lanes stride over the sample's non-zeros, the margin w.x is a wave reduction, then every lane
// updates its coordinates with fp64 atomics.  n_i and z_i are updated by device-scope atomicAdd (executed at
// the memory side, so exact across the 8 XCDs) and w_i is recomputed from the values the atomics returned:
// concurrent updates to one coordinate never lose a gradient.  Only the w_i a sample READS may be stale (the
// per-XCD L2s are not coherent) -- the Hogwild relaxation.  The reference has the same staleness: its margin is
// computed in flatMap1 (:396-420) before the feedback of earlier samples reaches flatMap2 (:423-485).  Exact
// when the samples in flight touch disjoint coordinates.  Opt-in (updateMode = HOGWILD); the sequential mode
// stays the default because it is run-to-run deterministic.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr int THREADS = 256;
constexpr int WAVES = THREADS / 64;

__device__ __forceinline__ double ld_relaxed(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(THREADS) void ftrl_hogwild_kernel(const int64_t* __restrict__ indptr,
                                                              const int32_t* __restrict__ idx,
                                                              const double* __restrict__ val,
                                                              const double* __restrict__ label, int64_t nrows,
                                                              double* w, double* n, double* z, double alpha,
                                                              double beta, double l1, double l2) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * WAVES;
    for (int64_t r = wave; r < nrows; r += nwaves) {
        const int64_t s = indptr[r], e = indptr[r + 1];
        double wx = 0.0;
        for (int64_t k = s + lane; k < e; k += 64) wx = fma(val[k], ld_relaxed(&w[idx[k]]), wx);
        for (int off = 32; off > 0; off >>= 1) wx += __shfl_xor(wx, off);
        const double p = 1.0 / (1.0 + exp(-wx));
        const double err = p - label[r];
        for (int64_t k = s + lane; k < e; k += 64) {
            const int32_t i = idx[k];
            const double g = err * val[k];
            const double g2 = g * g;
            const double wi = ld_relaxed(&w[i]);
            const double n_old = atomicAdd(&n[i], g2);
            const double n_new = n_old + g2;
            const double sigma = (sqrt(n_new) - sqrt(n_old)) / alpha;
            const double dz = g - sigma * wi;
            const double z_new = atomicAdd(&z[i], dz) + dz;
            const double wn = fabs(z_new) <= l1
                                  ? 0.0
                                  : ((z_new < 0 ? -1.0 : 1.0) * l1 - z_new) / (beta + sqrt(n_new) / alpha + l2);
            __hip_atomic_store(&w[i], wn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void ftrl_check_kernel(const int32_t* __restrict__ idx, int64_t nnz, int64_t dim, int* __restrict__ bad) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x)
        if (idx[k] < 0 || idx[k] >= dim) atomicOr(bad, 1);
}

}  // namespace

extern "C" {

// Validates every feature index against dim (bad[0] != 0 afterwards when one is out of range).  The caller runs
// it and checks bad before alink_ftrl_hogwild_f64: the update kernel trusts its indices.
int alink_ftrl_check_indices(const int32_t* idx, int64_t nnz, int64_t dim, int* bad, int grid, void* stream) {
    if (nnz <= 0) return 0;
    hipLaunchKernelGGL(ftrl_check_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), idx, nnz, dim, bad);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

int alink_ftrl_hogwild_f64(const int64_t* indptr, const int32_t* idx, const double* val, const double* label,
                           int64_t nrows, double* w, double* n, double* z, double alpha, double beta, double l1,
                           double l2, int grid, void* stream) {
    if (nrows <= 0) return 0;
    if (grid <= 0 || alpha <= 0.0) return 1;
    hipLaunchKernelGGL(ftrl_hogwild_kernel, dim3(grid), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                       indptr, idx, val, label, nrows, w, n, z, alpha, beta, l1, l2);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
