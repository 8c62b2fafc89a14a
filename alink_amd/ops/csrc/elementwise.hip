// Fused elementwise kernels on CDNA4 (gfx950 / MI355X): SURVEY §2.13 K6 (GBDT gradient / hessian statistics and
// the per-tree prediction update), K17 (MLP bias + sigmoid forward / sigmoid backward epilogues) and K27 (scaler / imputer / binarizer transforms of dense column blocks).
//
// All of these are pure HBM streams: one read of each operand and one write of the result, replacing chains of
// 5-12 torch elementwise launches (each re-reading and re-writing the whole column).  Arithmetic is done in the
// same order and precision as the torch reference so results are bit-identical: FP contraction is off for the
// file (no FMA fusing of ``(x - a) / b * c + e``).
//
// Reference behaviour:
//   K6  ConstructLocalBin g/h (A/operator/common/tree/parallelcart/ConstructLocalBin.java:116-131 least squares,
//       :185-205 logistic) and Split.java's predBuf update (pred += leaf mean, rounded to float).
//   K27 StandardScalerModelMapper / MinMaxScalerModelMapper / MaxAbsScalerModelMapper / ImputerModelMapper /
//       BinarizerMapper (A/operator/common/dataproc/*, A/operator/common/feature/BinarizerMapper.java).
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace {

constexpr int TB = 256;

inline int grid_for(int64_t work) {
  // grid-stride loops; 8 waves per CU worth of blocks on 256 CUs is enough to saturate HBM
  int64_t g = (work + TB - 1) / TB;
  return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

// ---------------------------------------------------------------------------------------------------------------
// K6: per-row GBDT statistics {g*g, g, h, 1} (float4, the histogram kernel's 16-B row record)
//   algo 0 (least squares): g = f - y, h = 1
//   algo 1 (logistic):      p = 1 / (1 + exp(-f)) in fp64, g = float(p - y), h = float(p (1 - p))
//   optional per-row weights multiply g and h (in fp32, after rounding, like the torch path)
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(TB) void gbdt_grad_stats_kernel(const float* __restrict__ pred,
                                                             const float* __restrict__ y,
                                                             const float* __restrict__ w, int64_t n, int algo,
                                                             float4* __restrict__ stats) {
  for (int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TB) {
    const float f = pred[i], yy = y[i];
    float g, h;
    if (algo == 1) {
      const double p = 1.0 / (1.0 + exp(-(double)f));
      g = (float)(p - (double)yy);
      h = (float)(p * (1.0 - p));
    } else {
      g = f - yy;
      h = 1.0f;
    }
    if (w != nullptr) {
      const float ww = w[i];
      g = g * ww;
      h = h * ww;
    }
    stats[i] = make_float4(g * g, g, h, 1.0f);
  }
}

// pred[i] = float(double(pred[i]) + vals[-1 - code[i]]) for rows that ended in a leaf (code < 0)
__global__ __launch_bounds__(TB) void gbdt_leaf_update_kernel(float* __restrict__ pred,
                                                              const int32_t* __restrict__ codes,
                                                              const double* __restrict__ vals, int nvals,
                                                              int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TB) {
    const int32_t c = codes[i];
    if (c < 0) {
      int leaf = -1 - c;
      leaf = leaf < nvals ? leaf : nvals - 1;
      pred[i] = (float)((double)pred[i] + vals[leaf]);
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K27: column-parameterised transform of a dense row-major block X[n, d] -> out[n, d] (fp64 out)
//   mode 0 standard:  b[j] > 0 ? (x - a[j]) / b[j] : 0
//   mode 1 min-max:   (b[j] - a[j]) != 0 ? (x - a[j]) / (b[j] - a[j]) * (hi - lo) + lo : 0.5 (hi + lo)
//   mode 2 max-abs:   a[j] == 0 ? x : x / a[j]
//   mode 3 impute:    isnan(x) ? a[j] : x
//   mode 4 binarize:  x > lo ? 1 : 0
// in_dtype 0 fp32, 1 fp64.  One thread per element (grid-stride); column index from the flat offset.
// ---------------------------------------------------------------------------------------------------------------
template <typename T, int MODE>
__global__ __launch_bounds__(TB) void col_transform_kernel(const T* __restrict__ X, int64_t total, int d,
                                                           const double* __restrict__ a,
                                                           const double* __restrict__ b, double lo, double hi,
                                                           double* __restrict__ out) {
  for (int64_t e = (int64_t)blockIdx.x * TB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TB) {
    const double x = (double)X[e];
    const int j = (int)(e % d);
    double r;
    if (MODE == 0) {
      const double s = b[j];
      r = s > 0.0 ? (x - a[j]) / s : 0.0;
    } else if (MODE == 1) {
      const double rng = b[j] - a[j];
      r = rng != 0.0 ? (x - a[j]) / rng * (hi - lo) + lo : 0.5 * (hi + lo);
    } else if (MODE == 2) {
      const double m = a[j];
      r = m == 0.0 ? x : x / m;
    } else if (MODE == 3) {
      r = x != x ? a[j] : x;
    } else {
      r = x > lo ? 1.0 : 0.0;
    }
    out[e] = r;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// K17: MLP hidden-layer epilogues around the hipBLASLt GEMMs
//   forward:  Z[i, j] = 1 / (1 + exp(-(Z[i, j] + b[j])))      (bias + sigmoid in place)
//   backward: G[i] *= S[i] (1 - S[i])                           (sigmoid derivative in place)
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(TB) void bias_sigmoid_kernel(double* __restrict__ Z, int64_t total, int d,
                                                          const double* __restrict__ b) {
  for (int64_t e = (int64_t)blockIdx.x * TB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TB) {
    const double z = Z[e] + b[e % d];
    Z[e] = 1.0 / (1.0 + exp(-z));
  }
}

__global__ __launch_bounds__(TB) void sigmoid_bwd_kernel(double* __restrict__ G, const double* __restrict__ S,
                                                         int64_t total) {
  for (int64_t e = (int64_t)blockIdx.x * TB + threadIdx.x; e < total; e += (int64_t)gridDim.x * TB) {
    const double s = S[e];
    G[e] = G[e] * (s * (1.0 - s));
  }
}

template <typename T>
hipError_t launch_transform(const void* X, int64_t total, int d, int mode, const double* a, const double* b,
                            double lo, double hi, double* out, hipStream_t s) {
  const dim3 grid(grid_for(total)), block(TB);
  const T* x = static_cast<const T*>(X);
  switch (mode) {
    case 0: hipLaunchKernelGGL((col_transform_kernel<T, 0>), grid, block, 0, s, x, total, d, a, b, lo, hi, out); break;
    case 1: hipLaunchKernelGGL((col_transform_kernel<T, 1>), grid, block, 0, s, x, total, d, a, b, lo, hi, out); break;
    case 2: hipLaunchKernelGGL((col_transform_kernel<T, 2>), grid, block, 0, s, x, total, d, a, b, lo, hi, out); break;
    case 3: hipLaunchKernelGGL((col_transform_kernel<T, 3>), grid, block, 0, s, x, total, d, a, b, lo, hi, out); break;
    case 4: hipLaunchKernelGGL((col_transform_kernel<T, 4>), grid, block, 0, s, x, total, d, a, b, lo, hi, out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

extern "C" {

int alink_gbdt_grad_stats(const void* pred, const void* y, const void* w, int64_t n, int algo, void* stats,
                          void* stream) {
  if (n <= 0) return 0;
  if (algo != 0 && algo != 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gbdt_grad_stats_kernel, dim3(grid_for(n)), dim3(TB), 0, (hipStream_t)stream,
                     (const float*)pred, (const float*)y, (const float*)w, n, algo, (float4*)stats);
  return (int)hipGetLastError();
}

int alink_gbdt_leaf_update(void* pred, const void* codes, const void* vals, int nvals, int64_t n, void* stream) {
  if (n <= 0) return 0;
  if (nvals <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gbdt_leaf_update_kernel, dim3(grid_for(n)), dim3(TB), 0, (hipStream_t)stream, (float*)pred,
                     (const int32_t*)codes, (const double*)vals, nvals, n);
  return (int)hipGetLastError();
}

int alink_bias_sigmoid_f64(void* Z, int64_t n, int d, const void* b, void* stream) {
  if (n <= 0 || d <= 0) return 0;
  const int64_t total = n * (int64_t)d;
  hipLaunchKernelGGL(bias_sigmoid_kernel, dim3(grid_for(total)), dim3(TB), 0, (hipStream_t)stream, (double*)Z, total,
                     d, (const double*)b);
  return (int)hipGetLastError();
}

int alink_sigmoid_bwd_f64(void* G, const void* S, int64_t total, void* stream) {
  if (total <= 0) return 0;
  hipLaunchKernelGGL(sigmoid_bwd_kernel, dim3(grid_for(total)), dim3(TB), 0, (hipStream_t)stream, (double*)G,
                     (const double*)S, total);
  return (int)hipGetLastError();
}

int alink_col_transform(const void* X, int64_t n, int d, int in_dtype, int mode, const void* a, const void* b,
                        double lo, double hi, void* out, void* stream) {
  if (n <= 0 || d <= 0) return 0;
  const int64_t total = n * (int64_t)d;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (in_dtype == 0)
    e = launch_transform<float>(X, total, d, mode, (const double*)a, (const double*)b, lo, hi, (double*)out, s);
  else if (in_dtype == 1)
    e = launch_transform<double>(X, total, d, mode, (const double*)a, (const double*)b, lo, hi, (double*)out, s);
  else
    e = hipErrorInvalidValue;
  return (int)e;
}

}  // extern "C"
