// Multinomial-logistic (softmax) loss epilogues on CDNA4 (gfx950 / MI355X): SURVEY §2.13 K16.
//
// The K-1 free logit columns eta = X W^T come from one hipBLASLt GEMM; everything after it is per-row work over
// k1 = K-1 values that torch runs as ~10 launches (cat a pivot zero, logsumexp, exp, nonzero + index_put of the
// label, multiply by the weight, and per line-search step again).  These kernels do it in one pass each:
//
//   softmax_grad:   R[i, j] = w_i (softmax_j(eta_i, 0) - [y_i == j]),  part[b] = sum_i w_i (lse_i - eta_i[y_i])
//                   (R feeds the X^T R gradient GEMM; class K-1 is the pivot with logit 0)
//   softmax_search: part[b, s] = sum_i w_i (lse(ec_i - s ed_i) - (ec_i - s ed_i)[y_i]) for s = 0..S
//                   (every trial step of the backtracking line search from one read of ec / ed)
//
// One thread per row with the k1 logits in registers (k1 <= KMAX, templated); per-block partial sums in fixed
// order (deterministic, no atomics), reduced on the host side.  Reference: SoftmaxObjFunc.java (calcLoss /
// updateGradient / calcSearchValues), A/operator/common/linear/SoftmaxObjFunc.java.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int TB = 256;
constexpr int WAVES = TB / 64;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block sum of v -> written by thread 0 to *dst; all threads must call
__device__ __forceinline__ void block_sum_store(double v, double* lds, double* dst) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) t += lds[i];
    *dst = t;
  }
  __syncthreads();
}

// log(exp(0) + sum_j exp(e_j)) with the pivot's zero logit included (max-shifted like torch.logsumexp)
template <int KMAX, bool PIVOT = true>
__device__ __forceinline__ double lse_pivot(const double (&e)[KMAX], int k1) {
  double m = PIVOT ? 0.0 : e[0];
#pragma unroll
  for (int j = 0; j < KMAX; ++j)
    if (j < k1) m = e[j] > m ? e[j] : m;
  double s = PIVOT ? exp(-m) : 0.0;
#pragma unroll
  for (int j = 0; j < KMAX; ++j)
    if (j < k1) s += exp(e[j] - m);
  return m + log(s);
}

template <int KMAX, bool PIVOT>
__global__ __launch_bounds__(TB) void softmax_grad_kernel(const double* __restrict__ eta,
                                                          const double* __restrict__ y,
                                                          const double* __restrict__ w, int64_t n, int k1,
                                                          double* __restrict__ R, double* __restrict__ part) {
  __shared__ double lds[WAVES];
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TB) {
    double e[KMAX];
    const double* row = eta + i * k1;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) e[j] = j < k1 ? row[j] : 0.0;
    const double lse = lse_pivot<KMAX, PIVOT>(e, k1);
    const int yk = (int)y[i];
    const double wi = w[i];
    double lin = 0.0;
    double* out = R + i * k1;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      if (j < k1) {
        double p = exp(e[j] - lse);
        if (j == yk) {
          lin = e[j];
          p -= 1.0;
        }
        out[j] = p * wi;
      }
    }
    acc += wi * (lse - lin);
  }
  block_sum_store(acc, lds, part + blockIdx.x);
}

template <int KMAX>
__global__ __launch_bounds__(TB) void softmax_search_kernel(const double* __restrict__ ec,
                                                            const double* __restrict__ ed,
                                                            const double* __restrict__ y,
                                                            const double* __restrict__ w, int64_t n, int k1,
                                                            double beta, int nsteps, double* __restrict__ part) {
  __shared__ double lds[WAVES];
  // steps processed in groups of 4 accumulators so the row's logits are read once per group (S+1 <= 64)
  for (int s0 = 0; s0 < nsteps; s0 += 4) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TB) {
      double c[KMAX], d[KMAX];
      const double* rc = ec + i * k1;
      const double* rd = ed + i * k1;
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        c[j] = j < k1 ? rc[j] : 0.0;
        d[j] = j < k1 ? rd[j] * beta : 0.0;
      }
      const int yk = (int)y[i];
      const double wi = w[i];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s = s0 + q;
        if (s < nsteps) {
          double e[KMAX];
          double lin = 0.0;
#pragma unroll
          for (int j = 0; j < KMAX; ++j) {
            e[j] = c[j] - (double)s * d[j];
            if (j == yk) lin = e[j];
          }
          acc[q] += wi * (lse_pivot<KMAX>(e, k1) - lin);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (s0 + q < nsteps) block_sum_store(acc[q], lds, part + (int64_t)blockIdx.x * nsteps + s0 + q);
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + TB - 1) / TB;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

}  // namespace

extern "C" {

// grid size the caller must size ``part`` for (blocks; search partials are [grid, nsteps])
int alink_softmax_grid(int64_t n) { return grid_for(n); }

int alink_softmax_grad_f64(const void* eta, const void* y, const void* w, int64_t n, int k1, void* R, void* part,
                           void* stream) {
  if (n <= 0) return 0;
  const dim3 grid(grid_for(n)), block(TB);
  hipStream_t s = (hipStream_t)stream;
  const double *e = (const double*)eta, *yy = (const double*)y, *ww = (const double*)w;
  double *r = (double*)R, *p = (double*)part;
  if (k1 <= 0) return (int)hipErrorInvalidValue;
  if (k1 <= 4) hipLaunchKernelGGL((softmax_grad_kernel<4, true>), grid, block, 0, s, e, yy, ww, n, k1, r, p);
  else if (k1 <= 16) hipLaunchKernelGGL((softmax_grad_kernel<16, true>), grid, block, 0, s, e, yy, ww, n, k1, r, p);
  else if (k1 <= 32) hipLaunchKernelGGL((softmax_grad_kernel<32, true>), grid, block, 0, s, e, yy, ww, n, k1, r, p);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// the same without a pivot class (all K logits free, labels in [0, K)): the MLP's softmax cross-entropy output layer
int alink_softmax_full_grad_f64(const void* z, const void* y, const void* w, int64_t n, int K, void* R, void* part,
                                void* stream) {
  if (n <= 0) return 0;
  const dim3 grid(grid_for(n)), block(TB);
  hipStream_t s = (hipStream_t)stream;
  const double *e = (const double*)z, *yy = (const double*)y, *ww = (const double*)w;
  double *r = (double*)R, *p = (double*)part;
  if (K <= 0) return (int)hipErrorInvalidValue;
  if (K <= 4) hipLaunchKernelGGL((softmax_grad_kernel<4, false>), grid, block, 0, s, e, yy, ww, n, K, r, p);
  else if (K <= 16) hipLaunchKernelGGL((softmax_grad_kernel<16, false>), grid, block, 0, s, e, yy, ww, n, K, r, p);
  else if (K <= 32) hipLaunchKernelGGL((softmax_grad_kernel<32, false>), grid, block, 0, s, e, yy, ww, n, K, r, p);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

int alink_softmax_search_f64(const void* ec, const void* ed, const void* y, const void* w, int64_t n, int k1,
                             double beta, int nsteps, void* part, void* stream) {
  if (n <= 0) return 0;
  if (k1 <= 0 || nsteps <= 0 || nsteps > 64) return (int)hipErrorInvalidValue;
  const dim3 grid(grid_for(n)), block(TB);
  hipStream_t s = (hipStream_t)stream;
  const double *c = (const double*)ec, *d = (const double*)ed, *yy = (const double*)y, *ww = (const double*)w;
  double* p = (double*)part;
  if (k1 <= 4) hipLaunchKernelGGL(softmax_search_kernel<4>, grid, block, 0, s, c, d, yy, ww, n, k1, beta, nsteps, p);
  else if (k1 <= 16)
    hipLaunchKernelGGL(softmax_search_kernel<16>, grid, block, 0, s, c, d, yy, ww, n, k1, beta, nsteps, p);
  else if (k1 <= 32)
    hipLaunchKernelGGL(softmax_search_kernel<32>, grid, block, 0, s, c, d, yy, ww, n, k1, beta, nsteps, p);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

}  // extern "C"
