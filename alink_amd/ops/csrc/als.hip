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

}  // extern "C"
