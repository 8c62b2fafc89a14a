// GMM E-step epilogue on CDNA4 (gfx950 / MI355X): SURVEY §2.13 K22.
//
// The Mahalanobis projections of every row onto every component come from ONE hipBLASLt GEMM,
// Z = X0 [n, d] @ [W_1 | ... | W_k] [d, k*d] (W_j = U_j diag(lambda^-1/2) the pseudo-inverse root of Sigma_j,
// X0 = X - global mean to keep the cancellation in z = x W_j - mu_j W_j small).  This kernel does the rest in one
// pass over Z: per component the squared norm |Z_j - C_j|^2 (C_j = (mu_j - xbar) W_j), the log density
// lp_j = cst_j - |.|^2 / 2 (cst_j folds -1/2 (rank_j log 2pi + logdet_j) + log w_j), the row's log-sum-exp and
// the responsibilities R[i, j] = exp(lp_j - lse).  Per-block sums of lse (the log-likelihood) in fixed order.
//
// One wave per row: lanes stride the d coordinates of a component (coalesced 512-B reads), a wave butterfly
// reduces each component's norm and lane j keeps lp_j (k <= 64).  Reference: GmmTrainBatchOp.java:174-214 and
// MultivariateGaussian.logpdf (A/common/probabilistic/..., A/operator/batch/clustering/GmmTrainBatchOp.java).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr int TB = 256;
constexpr int WAVES = TB / 64;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

__global__ __launch_bounds__(TB) void gmm_estep_kernel(const double* __restrict__ Z, int64_t n, int k, int d,
                                                       const double* __restrict__ C,
                                                       const double* __restrict__ cst, double* __restrict__ R,
                                                       double* __restrict__ part) {
  __shared__ double lds[WAVES];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t kd = (int64_t)k * d;
  double acc = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * WAVES + wid; row < n; row += (int64_t)gridDim.x * WAVES) {
    const double* z = Z + row * kd;
    double my = -INFINITY;
    for (int j = 0; j < k; ++j) {
      double s = 0.0;
      for (int t = lane; t < d; t += 64) {
        const double v = z[(int64_t)j * d + t] - C[(int64_t)j * d + t];
        s += v * v;
      }
      s = wave_sum(s);
      if (lane == j) my = cst[j] - 0.5 * s;
    }
    const double m = wave_max(my);
    const double e = lane < k ? exp(my - m) : 0.0;
    const double lse = m + log(wave_sum(e));
    if (lane < k) R[row * k + lane] = exp(my - lse);
    if (lane == 0) acc += lse;
  }
  // acc is only non-zero on lane 0 of each wave
  if (lane == 0) lds[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) t += lds[i];
    part[blockIdx.x] = t;
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + WAVES - 1) / WAVES;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

}  // namespace

extern "C" {

int alink_gmm_grid(int64_t n) { return grid_for(n); }

int alink_gmm_estep_f64(const void* Z, int64_t n, int k, int d, const void* C, const void* cst, void* R, void* part,
                        void* stream) {
  if (n <= 0) return 0;
  if (k <= 0 || k > 64 || d <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gmm_estep_kernel, dim3(grid_for(n)), dim3(TB), 0, (hipStream_t)stream, (const double*)Z, n, k,
                     d, (const double*)C, (const double*)cst, (double*)R, (double*)part);
  return (int)hipGetLastError();
}

}  // extern "C"
