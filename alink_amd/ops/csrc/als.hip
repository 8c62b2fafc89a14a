// ALS normal equations: for every row u of a CSR rating matrix
//   A_u = sum_t c_t * y_t y_t^T ,  b_u = sum_t w_t * y_t      (y_t = factors of the t-th neighbour)
// explicit feedback: c = 1, w = rating; implicit: c = alpha*r (r > 0), w = 1 + c (r > 0), else 0
// (reference: AlsTrain.UpdateFactorsFunc.coGroup AlsTrain.java:479-545 -> NormalEquation.add, dger/axpy).
//
// CDNA4 mapping: one 64-lane wavefront per row; the rank is padded to RP in {8,16,32,64}, and lane (li, lj)
// of an (RP/8) x (RP/8) lane grid owns an 8x8 register block of A_u.  Neighbour factors are staged through
// LDS 32 rows at a time (one coalesced sweep per tile), so each FMA costs 1/4 LDS read instead of 2.
// The host adds the regularisation (lambda * n_u, or lambda * #positive for implicit), the implicit
// Y^T Y term, and runs the batched Cholesky / NNLS solves.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kTile = 32;

template <int RP>
__global__ __launch_bounds__(64) void als_gram(const int64_t* __restrict__ indptr, const int32_t* __restrict__ nbr,
                                               const float* __restrict__ rating, const float* __restrict__ Y, int r,
                                               int implicit, float alpha, float* __restrict__ A,
                                               float* __restrict__ bvec) {
  constexpr int G = RP / 8;  // lane grid side
  __shared__ float tile[kTile][RP + 1];
  __shared__ float cw[kTile][2];
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x;
  const int li = lane / G, lj = lane % G;
  const bool active = lane < G * G;
  const int64_t s = indptr[row], e = indptr[row + 1];
  float acc[8][8];
  float bacc[8];
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    bacc[a] = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[a][c] = 0.f;
  }
  for (int64_t t0 = s; t0 < e; t0 += kTile) {
    const int cnt = (int)((e - t0) < kTile ? (e - t0) : kTile);
    for (int idx = lane; idx < kTile * RP; idx += 64) {
      const int t = idx / RP, k = idx - (idx / RP) * RP;
      float v = 0.f;
      if (t < cnt && k < r) v = Y[(int64_t)nbr[t0 + t] * r + k];
      tile[t][k] = v;
    }
    if (lane < kTile) {
      float c = 0.f, w = 0.f;
      if (lane < cnt) {
        const float rt = rating[t0 + lane];
        if (implicit) {
          c = rt > 0.f ? alpha * rt : 0.f;
          w = rt > 0.f ? 1.f + c : 0.f;
        } else {
          c = 1.f;
          w = rt;
        }
      }
      cw[lane][0] = c;
      cw[lane][1] = w;
    }
    __syncthreads();
    if (active) {
      for (int t = 0; t < cnt; ++t) {
        const float c = cw[t][0];
        float yi[8], yj[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          yi[a] = tile[t][li * 8 + a];
          yj[a] = tile[t][lj * 8 + a] * c;
        }
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int b = 0; b < 8; ++b) acc[a][b] = fmaf(yi[a], yj[b], acc[a][b]);
        if (lj == 0) {
          const float w = cw[t][1];
#pragma unroll
          for (int a = 0; a < 8; ++a) bacc[a] = fmaf(w, yi[a], bacc[a]);
        }
      }
    }
    __syncthreads();
  }
  if (!active) return;
  float* Au = A + row * (int64_t)r * r;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int i = li * 8 + a;
    if (i >= r) continue;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int j = lj * 8 + b;
      if (j < r) Au[i * r + j] = acc[a][b];
    }
    if (lj == 0) bvec[row * (int64_t)r + i] = bacc[a];
  }
}


// ---------------------------------------------------------------------------------------------------------------
// Fused ALS row solve (K11, the verdict's "one workgroup per system, in LDS"): for row u
//   A_u = sum_t c_t y_t y_t^T + reg_u I (+ Y^T Y, implicit),  b_u = sum_t w_t y_t,  x_u = A_u^{-1} b_u
// without materialising A_u in HBM (reference NormalEquation.java:44-92 + the per-user solve of
// AlsTrain.java:479-545).  One 64-lane wave per row, rank padded to RP:
//   1. Gram in registers, fp64: lane j owns column j; neighbour y_t is read coalesced (lane j <- y_t[j]) and
//      its entries are broadcast with v_readlane (y is fp32, so one readlane per entry), acc[i] += c y_i y_j;
//   2. the column is stored to LDS (column-major, stride RP+1), right-looking Cholesky with lane = row
//      (pivot broadcast from LDS, trailing update of the lane's row entries), fp64;
//   3. forward / backward substitution with lane = row, the running vector in a register and the pivot
//      element broadcast by v_readlane.  A non-positive pivot flags the row (status) for the host fallback.
// Padded dimensions carry an identity block, so their solution entries are 0.
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

template <int RP>
__global__ __launch_bounds__(64) void als_fused_solve(const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ nbr,
                                                      const float* __restrict__ rating, const float* __restrict__ Y,
                                                      int r, int implicit, float alpha, const double* __restrict__ reg,
                                                      const double* __restrict__ YtY, float* __restrict__ X,
                                                      int32_t* __restrict__ status) {
  constexpr int LD = RP + 1;
  __shared__ double S[RP * LD];
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t s = indptr[row], e = indptr[row + 1];
  double acc[RP];
#pragma unroll
  for (int i = 0; i < RP; ++i) acc[i] = 0.0;
  double bj = 0.0;
  for (int64_t t = s; t < e; ++t) {
    const float yf = lane < r ? Y[(int64_t)nbr[t] * r + lane] : 0.f;
    const float rt = rating[t];
    double c, w;
    if (implicit) {
      c = rt > 0.f ? (double)alpha * rt : 0.0;
      w = rt > 0.f ? 1.0 + c : 0.0;
    } else {
      c = 1.0;
      w = rt;
    }
    const double yj = yf;
    const double cy = c * yj;
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const float yi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yf), i));
      acc[i] = fma((double)yi, cy, acc[i]);
    }
    bj = fma(w, yj, bj);
  }
  // regularisation, implicit Y^T Y, identity on padded dimensions; column `lane` -> LDS.  Lanes >= RP
  // (RP < 64) own nothing: every LDS access below is guarded, their indices would alias other columns.
  const bool act = lane < RP;
  const double lam = reg[row];
#pragma unroll
  for (int i = 0; i < RP; ++i) {
    double v = acc[i];
    if (lane < r && i < r && YtY != nullptr) v += YtY[i * r + lane];
    if (i == lane) v += lane < r ? lam : 1.0;
    if (act) S[lane * LD + i] = v;
  }
  __syncthreads();
  // Cholesky A = L L^T, lane = row index; L overwrites the lower triangle (column k at S[k*LD + i])
  int bad = 0;
  for (int k = 0; k < RP; ++k) {
    const double d = S[k * LD + k];
    bad |= !(d > 0.0);
    const double piv = sqrt(d > 0.0 ? d : 1.0);
    const double inv = 1.0 / piv;
    double lik = 0.0;
    if (act && lane > k) {
      lik = S[k * LD + lane] * inv;
      S[k * LD + lane] = lik;
    }
    __syncthreads();
    if (lane == k) S[k * LD + k] = piv;
    for (int j = k + 1; j < RP; ++j) {
      const double ljk = S[k * LD + j];            // broadcast: L[j][k]
      if (act && lane >= j) S[j * LD + lane] -= lik * ljk;
    }
    __syncthreads();
  }
  // L z = b (lane = row), then L^T x = z
  double v = bj;
  for (int k = 0; k < RP; ++k) {
    const double zk = readlane_f64(v, k) / S[k * LD + k];
    if (act && lane > k) v -= S[k * LD + lane] * zk;
    if (lane == k) v = zk;
  }
  for (int k = RP - 1; k >= 0; --k) {
    const double xk = readlane_f64(v, k) / S[k * LD + k];
    if (lane < k) v -= S[lane * LD + k] * xk;
    if (lane == k) v = xk;
  }
  if (lane < r) X[row * r + lane] = (float)v;
  if (lane == 0) status[row] = bad;
}

}  // namespace

extern "C" {

// indptr [m+1] int64, nbr [nnz] int32 (row index into Y), rating [nnz] fp32, Y [n, r] fp32;
// A [m, r, r] and b [m, r] fp32 outputs (fully written).  r <= 64.
int alink_als_gram_f32(const int64_t* indptr, const int32_t* nbr, const float* rating, const float* Y, int64_t m,
                       int r, int implicit, float alpha, float* A, float* b, hipStream_t stream) {
  if (m <= 0) return 0;
  if (r <= 0 || r > 64) return 1;
  const dim3 grid((unsigned)m), block(64);
  if (r <= 8)
    hipLaunchKernelGGL(als_gram<8>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, A, b);
  else if (r <= 16)
    hipLaunchKernelGGL(als_gram<16>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, A, b);
  else if (r <= 32)
    hipLaunchKernelGGL(als_gram<32>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, A, b);
  else
    hipLaunchKernelGGL(als_gram<64>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, A, b);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Fused normal equations + Cholesky solve per row: X [m, r] fp32 out, status [m] (non-zero: not SPD -> the
// caller re-solves that row).  reg [m] fp64 = lambda * n_u; YtY [r, r] fp64 (implicit) or null.  r <= 64.
int alink_als_fused_solve(const int64_t* indptr, const int32_t* nbr, const float* rating, const float* Y, int64_t m,
                          int r, int implicit, float alpha, const double* reg, const double* YtY, float* X,
                          int32_t* status, hipStream_t stream) {
  if (m <= 0) return 0;
  if (r <= 0 || r > 64) return 1;
  const dim3 grid((unsigned)m), block(64);
  if (r <= 8)
    hipLaunchKernelGGL(als_fused_solve<8>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, reg,
                       YtY, X, status);
  else if (r <= 16)
    hipLaunchKernelGGL(als_fused_solve<16>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, reg,
                       YtY, X, status);
  else if (r <= 32)
    hipLaunchKernelGGL(als_fused_solve<32>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, reg,
                       YtY, X, status);
  else
    hipLaunchKernelGGL(als_fused_solve<64>, grid, block, 0, stream, indptr, nbr, rating, Y, r, implicit, alpha, reg,
                       YtY, X, status);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
