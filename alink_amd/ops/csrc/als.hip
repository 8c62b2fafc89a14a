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
  // fp32 FMAs within a 32-neighbour tile, tile partials folded into fp64 so high-degree rows (popular items,
  // ~1e5 neighbours) keep fp64-level accuracy like the torch path (normal_equations_torch accumulates in fp64)
  double dacc[8][8];
  double dbacc[8];
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    dbacc[a] = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) dacc[a][c] = 0.0;
  }
  for (int64_t t0 = s; t0 < e; t0 += kTile) {
    float acc[8][8];
    float bacc[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      bacc[a] = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[a][c] = 0.f;
    }
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
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        dbacc[a] += (double)bacc[a];
#pragma unroll
        for (int b = 0; b < 8; ++b) dacc[a][b] += (double)acc[a][b];
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
      if (j < r) Au[i * r + j] = (float)dacc[a][b];
    }
    if (lj == 0) bvec[row * (int64_t)r + i] = (float)dbacc[a];
  }
}


// ---------------------------------------------------------------------------------------------------------------
// Fused ALS row solve (K11, the verdict's "one workgroup per system, in LDS"): for row u
//   A_u = sum_t c_t y_t y_t^T + reg_u I (+ Y^T Y, implicit),  b_u = sum_t w_t y_t,  x_u = A_u^{-1} b_u
// without materialising A_u in HBM (reference NormalEquation.java:44-92 + the per-user solve of
// AlsTrain.java:479-545).  One 64-lane wave per row, rank padded to RP:
//   1. Gram in registers, fp64: lane j owns column j; neighbour y_t is read coalesced (lane j <- y_t[j]) and
//      its entries are broadcast with v_readlane (y is fp32, so one readlane per entry), acc[i] += c y_i y_j;
//   2. right-looking Cholesky with lane = row entirely in registers (the symmetric Gram column is the row),
//      pivots and L[j][k] broadcast from their owner lanes by v_readlane, loops fully unrolled so every
//      register index is static; no LDS, so occupancy is set by the ~2 x RP fp64 registers alone;
//   3. forward / backward substitution the same way.  A non-positive pivot flags the row (status) for the
//      host fallback.
// Padded dimensions carry an identity block, so their solution entries are 0.
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// Cholesky + both substitutions in registers, lane = row: a[j] = A[lane][j] (symmetric), v = b[lane].  After the
// call v holds x[lane]; returns non-zero when a pivot was not positive.  Pivots and L[j][k] come from their
// owner lanes by v_readlane; loops fully unrolled, so every register index is static (no LDS, no scratch).
template <int RP>
__device__ __forceinline__ int chol_solve_regs(double (&a)[RP], double& v, int lane) {
  int bad = 0;
#pragma unroll
  for (int k = 0; k < RP; ++k) {
    const double d = readlane_f64(a[k], k);
    bad |= !(d > 0.0);
    const double piv = sqrt(d > 0.0 ? d : 1.0);
    const double lik = a[k] * (1.0 / piv);
#pragma unroll
    for (int j = k + 1; j < RP; ++j) a[j] -= lik * readlane_f64(lik, j);
    a[k] = lane > k ? lik : (lane == k ? piv : a[k]);
  }
  // L z = b: lane i subtracts L[i][k] z_k (its own a[k]) for k < i
#pragma unroll
  for (int k = 0; k < RP; ++k) {
    const double zk = readlane_f64(v, k) / readlane_f64(a[k], k);
    v = lane > k ? v - a[k] * zk : (lane == k ? zk : v);
  }
  // L^T x = z: x_k final, lanes i < k subtract L[k][i] x_k (L[k][i] = lane k's a[i])
#pragma unroll
  for (int k = RP - 1; k >= 0; --k) {
    const double xk = readlane_f64(v, k) / readlane_f64(a[k], k);
    if (lane == k) v = xk;
#pragma unroll
    for (int i = 0; i < k; ++i) {
      const double lki = readlane_f64(a[i], k);
      if (lane == i) v -= lki * xk;
    }
  }
  return bad;
}

// Gram of neighbours [s, e) of one row into the lane's column (lane j: a[i] += c y_i y_j, v += w y_j)
template <int RP>
__device__ __forceinline__ void gram_regs(const int32_t* __restrict__ nbr, const float* __restrict__ rating,
                                          const float* __restrict__ Y, int r, int implicit, float alpha, int64_t s,
                                          int64_t e, int lane, double (&a)[RP], double& v) {
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
    const double cy = c * (double)yf;
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const float yi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yf), i));
      a[i] = fma((double)yi, cy, a[i]);
    }
    v = fma(w, (double)yf, v);
  }
}

template <int RP>
__device__ __forceinline__ void add_reg(double (&a)[RP], int lane, int r, double lam, const double* __restrict__ YtY) {
#pragma unroll
  for (int i = 0; i < RP; ++i) {
    if (lane < r && i < r && YtY != nullptr) a[i] += YtY[i * r + lane];
    if (i == lane) a[i] += lane < r ? lam : 1.0;   // padded dimensions: identity
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Light rows, v2: one 64-lane wave per row, lane i = row i of the system, four rows per 256-thread workgroup.
//   Gram:  the neighbour factors are loaded 8 rows at a time (one coalesced fp32 load per lane each), staged as
//          fp64 in the wave's LDS slice and read back as broadcast ds_read_b128 pairs: a_i[j] += c_t y_i y_j is
//          one fp64 FMA per entry with no cross-lane moves (v1 paid two v_readlane per entry).
//   Solve: Gauss-Jordan elimination WITHOUT pivoting on the SPD system (the trailing block stays symmetric, so
//          the pivot row's trailing part equals the pivot column: one ds_write_b64 per lane broadcasts it).  Every
//          lane i != k eliminates column k from its row (a_i[j] -= (a_i[k]/a_kk) a_k[j], j > k) and its rhs; after
//          RP steps the system is diagonal and x_i = v_i / a_ii — no back substitution, no per-entry readlane
//          chain (v1's register Cholesky ran at 1 wave per SIMD, latency-bound on v_readlane hazards).
//   Precision: fp64 throughout (reference NormalEquation + LAPACK dposv are fp64).  A non-positive pivot flags
//   the row for the host pinv fallback.
// ---------------------------------------------------------------------------------------------------------------
constexpr int GJ_WAVES = 4;
constexpr int GJ_NB = 16;    // LDS rows per wave (neighbour staging, two batches of 8; the GJ pivot rows use 0-1)

template <int RP>
__device__ __forceinline__ void lds_wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// a[j] += coef * buf[j] for j in [j0, RP) (j0 and RP compile-time after unrolling): broadcast ds_read_b128 in
// batches of 8 entries, the next batch's reads issued before this batch's FMAs, scheduling fences between batches
// (at most 32 VGPRs of reads in flight next to the 2*RP of the row)
template <int RP>
__device__ __forceinline__ void axpy_bcast(double (&a)[RP], double coef, const double* buf, int j0) {
  constexpr int NB = 8;
  const int jb0 = j0 & ~(NB - 1);
  double2 q[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) q[u] = *reinterpret_cast<const double2*>(buf + jb0 + 2 * u);
#pragma unroll
  for (int jb = 0; jb < RP; jb += NB) {
    if (jb < jb0) continue;
    double2 n[4];
    if (jb + NB < RP) {
#pragma unroll
      for (int u = 0; u < 4; ++u) n[u] = *reinterpret_cast<const double2*>(buf + jb + NB + 2 * u);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // the empty volatile asm pins each update here: without it the compiler defers updates of far columns
      // to their use, keeping every step's broadcast values live (hundreds of VGPRs, scratch spills)
      if (jb + 2 * u >= j0) {
        a[jb + 2 * u] = fma(coef, q[u].x, a[jb + 2 * u]);
        asm volatile("" : "+v"(a[jb + 2 * u]));
      }
      if (jb + 2 * u + 1 >= j0) {
        a[jb + 2 * u + 1] = fma(coef, q[u].y, a[jb + 2 * u + 1]);
        asm volatile("" : "+v"(a[jb + 2 * u + 1]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (jb + NB < RP) {
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = n[u];
    }
  }
}

// Gram of neighbours [s, e) for one row, lane i = row i (a[j] += c y_i y_j, v += w y_i): neighbours are gathered
// GB_ROWS at a time (one coalesced fp32 row load per lane each, the next batch's loads issued before this batch's
// FMAs, so a wave keeps GB_ROWS rows in flight instead of one), staged as fp64 in one of two LDS batches and read
// back as broadcast pairs.  Branch-free: past-the-end neighbours load a valid row and get weight 0 (a guarded load
// or a guarded axpy makes the compiler copy the whole register row at every join).
constexpr int GB_ROWS = 8;

template <int RP>
__device__ __forceinline__ void gram_lds(const int32_t* __restrict__ nbr, const float* __restrict__ rating,
                                         const float* __restrict__ Y, int r, int implicit, float alpha, int64_t s,
                                         int64_t e, int lane, double (&a)[RP], double& v, double* buf) {
  if (s >= e) return;
  const int col = lane < r ? lane : r - 1;
  float yn[GB_ROWS];
#pragma unroll
  for (int u = 0; u < GB_ROWS; ++u) {
    const int64_t t = s + u < e ? s + u : e - 1;
    yn[u] = Y[(int64_t)nbr[t] * r + col];
  }
  int nb = 0;
  for (int64_t t0 = s; t0 < e; t0 += GB_ROWS, ++nb) {
    float yc[GB_ROWS];
#pragma unroll
    for (int u = 0; u < GB_ROWS; ++u) yc[u] = lane < r ? yn[u] : 0.f;
#pragma unroll
    for (int u = 0; u < GB_ROWS; ++u) {   // next batch (clamped: the last batch reloads row e - 1)
      const int64_t t = t0 + GB_ROWS + u < e ? t0 + GB_ROWS + u : e - 1;
      yn[u] = Y[(int64_t)nbr[t] * r + col];
    }
    double* rows = buf + (nb & 1) * (GB_ROWS * 64);
#pragma unroll
    for (int u = 0; u < GB_ROWS; ++u) rows[u * 64 + lane] = (double)yc[u];
    lds_wave_sync<RP>();
#pragma unroll
    for (int u = 0; u < GB_ROWS; ++u) {
      const bool live = t0 + u < e;
      const float rt = rating[live ? t0 + u : e - 1];
      double c, w;
      if (implicit) {
        c = rt > 0.f ? (double)alpha * rt : 0.0;
        w = rt > 0.f ? 1.0 + c : 0.0;
      } else {
        c = 1.0;
        w = rt;
      }
      c = live ? c : 0.0;
      w = live ? w : 0.0;
      axpy_bcast<RP>(a, c * (double)yc[u], rows + u * 64, 0);
      v = fma(w, (double)yc[u], v);
    }
  }
  lds_wave_sync<RP>();
}

// 1 / p to ~1 ulp: v_rcp_f64 + two Newton steps (the IEEE division sequence is ~4x longer and sits on the
// step's dependence chain)
__device__ __forceinline__ double rcp_f64(double p) {
  double r = __builtin_amdgcn_rcp(p);
  r = fma(fma(-p, r, 1.0), r, r);
  r = fma(fma(-p, r, 1.0), r, r);
  return r;
}

// Gauss-Jordan on the SPD system in registers (lane = row), pivot columns broadcast through two alternating LDS
// rows; after the last step v = x_i.  Software-pipelined across steps: step K updates column K+1 first and
// writes it to the other row immediately, so the LDS write -> read latency of step K+1's broadcast overlaps the
// rest of step K's row update (and no trailing wait is needed: step K+1 starts with the wait that also retires
// step K's reads before anything overwrites their row).  One step per template instance (K compile-time: every
// register index static; a 64-step `#pragma unroll` loop exceeds the unroller's size limit and would fall back to
// scratch-indexed arrays).
template <int RP, int K>
struct GJStep {
  static __device__ __forceinline__ void run(double (&a)[RP], double& v, double& diag, int& bad, int lane,
                                             double* buf) {
    __builtin_amdgcn_sched_barrier(0);   // one step at a time: keeps the register pressure at a[] + a few
    double* cur = buf + (K & 1) * 64;    // column K (written by step K-1, or before step 0)
    double* nxt = buf + ((K + 1) & 1) * 64;
    lds_wave_sync<RP>();
    const double p = readlane_f64(a[K], K);
    const double vk = readlane_f64(v, K);
    bad |= !(p > 0.0);
    const double rp = rcp_f64(p > 0.0 ? p : 1.0);
    const double f = lane == K ? 0.0 : a[K] * rp;
    diag = lane == K ? p : diag;
    if constexpr (K + 1 < RP) {
      a[K + 1] = fma(-f, cur[K + 1], a[K + 1]);
      asm volatile("" : "+v"(a[K + 1]));
      nxt[lane] = a[K + 1];              // next step's pivot column, in flight during the rest of this step
      if constexpr (K + 2 < RP) axpy_bcast<RP>(a, -f, cur, K + 2);   // a_i[j] -= f_i a_K[j], j > K + 1
    }
    v = fma(-f, vk, v);
    if constexpr (K + 1 < RP) GJStep<RP, K + 1>::run(a, v, diag, bad, lane, buf);
  }
};

template <int RP>
__device__ __forceinline__ int gj_solve(double (&a)[RP], double& v, int lane, double* buf) {
  int bad = 0;
  double diag = 1.0;
  lds_wave_sync<RP>();                   // the Gram phase's last reads of buf are done
  buf[lane] = a[0];
  GJStep<RP, 0>::run(a, v, diag, bad, lane, buf);
  lds_wave_sync<RP>();
  v = v / (diag > 0.0 ? diag : 1.0);
  return bad;
}

template <int RP>
__global__ __launch_bounds__(64 * GJ_WAVES) void als_fused_solve(const int64_t* __restrict__ indptr,
                                                                 const int32_t* __restrict__ nbr,
                                                                 const float* __restrict__ rating,
                                                                 const float* __restrict__ Y, int r, int implicit,
                                                                 float alpha, const double* __restrict__ reg,
                                                                 const double* __restrict__ YtY,
                                                                 const int64_t* __restrict__ rows, int64_t nrows,
                                                                 float* __restrict__ X, int32_t* __restrict__ status) {
  // every lane writes its own entry (64 per row, whatever RP is): rows of 64 doubles
  __shared__ __attribute__((aligned(16))) double lbuf[GJ_WAVES][GJ_NB * 64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform row bounds -> scalar loads
  const int lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * GJ_WAVES + w;
  if (idx >= nrows) return;              // whole wave: no block-wide barrier below
  const int64_t row = rows != nullptr ? rows[idx] : idx;
  double* buf = lbuf[w];
  double a[RP];
#pragma unroll
  for (int i = 0; i < RP; ++i) a[i] = 0.0;
  double v = 0.0;
  gram_lds<RP>(nbr, rating, Y, r, implicit, alpha, indptr[row], indptr[row + 1], lane, a, v, buf);
  add_reg<RP>(a, lane, r, reg[row], YtY);
  const int bad = gj_solve<RP>(a, v, lane, buf);
  if (lane < r) X[row * r + lane] = (float)v;
  if (lane == 0) status[row] = bad;
}

// ---------------------------------------------------------------------------------------------------------------
// Light rows on the matrix cores (rank 33..64, RP = 64): the whole normal-equation solve in v_mfma_f64_16x16x4
// C-layout tiles, fp64 throughout, no LDS.
//   Basis: the system is formed in the permuted order p = 16 I + m  <->  column j = 4 m + I, so that lane
//   (k = lane >> 4, m = lane & 15) of a 4-neighbour step loads columns 4m .. 4m+3 of neighbour k with ONE
//   16-byte load and holds exactly the MFMA operands: A operand of tile row I = c_k y_k[4m + I], B operand of
//   tile column J = y_k[4m + J].  Gram: 10 upper tiles (I <= J) += A_I x B_J per step (10 MFMAs per 4
//   neighbours, no cross-lane traffic: the r2 VALU Gram broadcast every neighbour through LDS and was bound by
//   LDS bandwidth, profiles/als_r3.txt).
//   Solve: block LDL^T over the 4 x 4 tile grid.  A C-layout tile S (lane: column lane & 15, rows
//   (lane >> 4) + 4 s in register s) is, register by register, the B operand of S and the A operand of S^T
//   (checked by tools/micro/mfma_f64_probe.hip), so every product below is "S^T x T" with both tiles straight
//   from registers:
//     D_k^-1       sweep operator on the 16 x 16 diagonal tile (cross-lane reads by __shfl; SPD, no pivoting;
//                  D^-1 is symmetric, so its C-layout also serves as its own A operand; the sweep leaves -D^-1,
//                  which the products below use as is, so no operand is ever negated);
//     W_kj = D_k^-1 A_kj;  A_ij -= A_ki^T W_kj  (k < i <= j);  V_kj = A_kj^T D_k^-1 (kept for the back
//     substitution) -- 88 MFMAs per system;
//   the vector steps z_k = D_k^-1 b_k, b_i -= A_ki^T z_k, x_k = z_k - sum_j V_kj^T x_j run on the VALU with one
//   vector entry per lane (tvec: __shfl gathers, 4 FMAs, two xor-shuffle reductions).
// A non-positive pivot flags the row for the host pinv fallback, as in the other paths.
// ---------------------------------------------------------------------------------------------------------------
typedef double d4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4_t mf64(double a, double b, d4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// acc + S^T x T (sgn = +1) or acc - S^T x T (sgn = -1)
template <int SGN>
__device__ __forceinline__ d4_t mm_tn(const d4_t& S, const d4_t& T, d4_t acc) {
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = mf64(SGN > 0 ? S[s] : -S[s], T[s], acc);
  return acc;
}

__device__ __forceinline__ d4_t mm_tn0(const d4_t& S, const d4_t& T) {
  d4_t z = {0.0, 0.0, 0.0, 0.0};
  return mm_tn<1>(S, T, z);
}

// vectors: one entry per lane, v[p] at lane p (segment q = entries 16q .. 16q+15).  T^T v_k for a C-layout tile
// T and segment k: lane (g, m) takes v_k[g + 4s] by __shfl, sums T[g + 4s][m] v_k[g + 4s] over its 4 rows and the
// partials over g by two xor shuffles -> (T^T v_k)[m] on every lane with column m.
__device__ __forceinline__ double tvec(const d4_t& T, double v, int k, int g) {
  double u = 0.0;
#pragma unroll
  for (int s = 0; s < 4; ++s) u = fma(T[s], __shfl(v, 16 * k + g + 4 * s), u);
  u += __shfl_xor(u, 16);
  u += __shfl_xor(u, 32);
  return u;
}

// -D^-1 of an SPD 16 x 16 C-layout tile by 16 sweep steps (after sweeping every index the matrix is -D^-1)
__device__ __forceinline__ d4_t sweep_neg_inv16(d4_t a, int lane, int& bad) {
  const int g = lane >> 4, j = lane & 15;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int kr = k >> 2, kg = k & 3;
    const double d = __shfl(a[kr], 16 * kg + k);                // D[k][k]
    const double row = __shfl(a[kr], 16 * kg + j);              // D[k][j]
    double col[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) col[s] = __shfl(a[s], 16 * g + k);   // D[g + 4s][k]
    bad |= !(d > 0.0);
    const double rd = rcp_f64(d > 0.0 ? d : 1.0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int i = g + 4 * s;
      double v = fma(-col[s] * rd, row, a[s]);
      v = j == k ? col[s] * rd : v;
      v = i == k ? row * rd : v;
      v = (i == k && j == k) ? -rd : v;
      a[s] = v;
    }
  }
  return a;
}

constexpr int MF_WAVES = 4;

__host__ __device__ constexpr int ut(int I, int J) { return I * 4 - I * (I - 1) / 2 + (J - I); }   // upper tile id

template <bool VEC4, bool IMPL>
__global__ __launch_bounds__(64 * MF_WAVES, 3) void als_mfma_solve(const int64_t* __restrict__ indptr,
                                                                const int32_t* __restrict__ nbr,
                                                                const float* __restrict__ rating,
                                                                const float* __restrict__ Y, int r, float alpha,
                                                                const double* __restrict__ reg,
                                                                const double* __restrict__ YtY,
                                                                const int64_t* __restrict__ rows, int64_t nrows,
                                                                float* __restrict__ X, int32_t* __restrict__ status) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * MF_WAVES + w;
  if (idx >= nrows) return;                       // whole wave; no block barrier below
  const int64_t row = rows != nullptr ? rows[idx] : idx;
  const int g = lane >> 4, m = lane & 15;
  const bool colok = VEC4 ? 4 * m < r : true;
  // tiles start as reg I (+ Y^T Y for implicit feedback); padded dimensions get an identity block
  d4_t A[10];
  const double lam = reg[row];
#pragma unroll
  for (int I = 0; I < 4; ++I)
#pragma unroll
    for (int J = I; J < 4; ++J)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int mi = g + 4 * q;                  // row inside the tile (column: m)
        const int ji = 4 * mi + I, jj = 4 * m + J; // original indices
        double add = 0.0;
        if (IMPL && YtY != nullptr && ji < r && jj < r) add = YtY[ji * r + jj];
        if (I == J && mi == m) add += ji < r ? lam : 1.0;
        A[ut(I, J)][q] = add;
      }
  double bacc[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t s = indptr[row], e = indptr[row + 1];
  if (e > s) {
    auto load_y = [&](int64_t nb, float (&y)[4]) {
      if (VEC4) {
        if (colok) {
          const float4 q = *reinterpret_cast<const float4*>(Y + nb * r + 4 * m);
          y[0] = q.x; y[1] = q.y; y[2] = q.z; y[3] = q.w;
        } else {
          y[0] = y[1] = y[2] = y[3] = 0.f;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = 4 * m + q < r ? Y[nb * r + 4 * m + q] : 0.f;
      }
    };
    // one step ahead: factors of the next 4 neighbours and the neighbour ids after them are in flight while this
    // step's 10 MFMAs run (past-the-end neighbours reload row e - 1 and get weight 0)
    int64_t tc = s + g < e ? s + g : e - 1;
    float ycur[4];
    load_y(nbr[tc], ycur);
    float rcur = rating[tc];
    int64_t tn = s + 4 + g < e ? s + 4 + g : e - 1;
    int32_t nbn = nbr[tn];
    float rn = rating[tn];
    for (int64_t t0 = s; t0 < e; t0 += 4) {
      float ynext[4];
      load_y(nbn, ynext);
      const float rnext = rn;
      const int64_t t2 = t0 + 8 + g < e ? t0 + 8 + g : e - 1;
      nbn = nbr[t2];
      rn = rating[t2];
      const bool live = t0 + g < e;
      double cw, ww;
      if (IMPL) {
        cw = rcur > 0.f ? (double)alpha * rcur : 0.0;
        ww = rcur > 0.f ? 1.0 + cw : 0.0;
      } else {
        cw = 1.0;
        ww = rcur;
      }
      cw = live ? cw : 0.0;
      ww = live ? ww : 0.0;
      double yb[4], ya[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        yb[q] = (double)ycur[q];
        ya[q] = cw * yb[q];
        bacc[q] = fma(ww, yb[q], bacc[q]);
      }
#pragma unroll
      for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = I; J < 4; ++J) A[ut(I, J)] = mf64(ya[I], yb[J], A[ut(I, J)]);
#pragma unroll
      for (int q = 0; q < 4; ++q) ycur[q] = ynext[q];
      rcur = rnext;
    }
  }
  // right-hand side b'[p] at lane p: lane (g, m) holds partials of b'[16 q + m] for its neighbour g
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bacc[q] += __shfl_xor(bacc[q], 16);
    bacc[q] += __shfl_xor(bacc[q], 32);
  }
  double v = g == 0 ? bacc[0] : g == 1 ? bacc[1] : g == 2 ? bacc[2] : bacc[3];
  // block LDL^T; the vector steps (z_k = D^-1 b_k, b_i -= A_ki^T z_k) run on the VALU between the tile products
  int bad = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const d4_t Dn = sweep_neg_inv16(A[ut(k, k)], lane, bad);      // -D_k^-1 (symmetric)
    const double z = -tvec(Dn, v, k, g);
    v = g == k ? z : v;
#pragma unroll
    for (int i = k + 1; i < 4; ++i) {
      const double u = tvec(A[ut(k, i)], v, k, g);
      v = g == i ? v - u : v;
    }
#pragma unroll
    for (int j = k + 1; j < 4; ++j) {
      const d4_t Wn = mm_tn0(Dn, A[ut(k, j)]);                      // -W_kj = -D^-1 A_kj
#pragma unroll
      for (int i = k + 1; i <= j; ++i) A[ut(i, j)] = mm_tn<1>(A[ut(k, i)], Wn, A[ut(i, j)]);
    }
#pragma unroll
    for (int j = k + 1; j < 4; ++j) A[ut(k, j)] = mm_tn0(A[ut(k, j)], Dn);   // -V_kj = -A_kj^T D^-1
  }
  // back substitution x_k = z_k - sum_{j > k} V_kj^T x_j  (the tiles hold -V_kj)
#pragma unroll
  for (int k = 2; k >= 0; --k) {
    double u = 0.0;
#pragma unroll
    for (int j = k + 1; j < 4; ++j) u += tvec(A[ut(k, j)], v, j, g);
    v = g == k ? v + u : v;
  }
  // x'[p] at lane p = 16 q + m -> original index 4 m + q
  {
    const int jo = 4 * m + g;
    if (jo < r) X[row * r + jo] = (float)v;
  }
  if (lane == 0) status[row] = bad;
}

// ---------------------------------------------------------------------------------------------------------------
// Explicit-feedback rows with few neighbours (m <= P < RP): the push-through identity
//     (Y_u^T Y_u + reg I_r)^{-1} Y_u^T r_u  =  Y_u^T (Y_u Y_u^T + reg I_m)^{-1} r_u
// turns the r x r system into an m x m one (padded to P with an identity block).  A user with 10 ratings at rank
// 64 solves 16 Gauss-Jordan steps over 16 columns instead of 64 over 64 (the r x r path is LDS-broadcast bound,
// see profiles/als_r3.txt).  One wave per row, lane = (i, q): row i = lane % P of the small system, k-chunk
// q = lane / P of the rank for the Gram; the Q = 64 / P partial dot products are summed with xor shuffles, then
// the same Gauss-Jordan as the r x r path (gj_solve<P>), then x = Y_u^T a with lane = rank entry.  fp64 throughout;
// the reference solves the r x r normal equations (NormalEquation.java:44-92) — the solutions agree to fp64
// rounding.  m > P flags the row for the host fallback.
// ---------------------------------------------------------------------------------------------------------------
constexpr int WB_WAVES = 4;
constexpr int WB_LD = 66;    // LDS row stride (doubles) of the staged factors

template <int P>
__global__ __launch_bounds__(64 * WB_WAVES) void als_woodbury_solve(const int64_t* __restrict__ indptr,
                                                                    const int32_t* __restrict__ nbr,
                                                                    const float* __restrict__ rating,
                                                                    const float* __restrict__ Y, int r,
                                                                    const double* __restrict__ reg,
                                                                    const int64_t* __restrict__ rows, int64_t nrows,
                                                                    float* __restrict__ X,
                                                                    int32_t* __restrict__ status) {
  constexpr int Q = 64 / P;
  constexpr int KC = 64 / Q;
  __shared__ __attribute__((aligned(16))) double ybuf[WB_WAVES][P * WB_LD];
  __shared__ __attribute__((aligned(16))) double gbuf[WB_WAVES][2 * 64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: every branch on m is scalar
  const int lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * WB_WAVES + w;
  if (idx >= nrows) return;              // whole wave: no block-wide barrier below
  const int64_t row = rows[idx];
  const int64_t s = indptr[row];
  const int64_t deg = indptr[row + 1] - s;
  const int m = __builtin_amdgcn_readfirstlane(deg > P ? 0 : (int)deg);
  double* yb = ybuf[w];
  // stage Y_u (fp32 -> fp64), rows t >= m zero; all P loads issued before the stores
  const int nb = lane < m ? nbr[s + lane] : 0;
  float yv[P];
#pragma unroll
  for (int t = 0; t < P; ++t) {
    // branch-free and traffic-free padding: a buffer resource over row it with 0 records for t >= m (and lanes
    // >= r past the record end) returns 0 without touching memory (a guarded load would make the compiler copy
    // arrays at every join; a clamped one would fetch P - m dead rows)
    const int it = __builtin_amdgcn_readlane(nb, t);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Y + (int64_t)it * r), (short)0, t < m ? r * 4 : 0, 0x00020000);
    yv[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
  }
#pragma unroll
  for (int t = 0; t < P; ++t) yb[t * WB_LD + lane] = (double)yv[t];
  lds_wave_sync<P>();
  // Gram K = Y_u Y_u^T: lane (i, q) sums entries [q KC, (q + 1) KC) of y_i . y_j, then xor-reduce over q
  const int i = lane % P;
  const int q = lane / P;
  double yi[KC];
#pragma unroll
  for (int k = 0; k < KC; k += 2) {
    const double2 t2 = *reinterpret_cast<const double2*>(yb + i * WB_LD + q * KC + k);
    yi[k] = t2.x;
    yi[k + 1] = t2.y;
  }
  double a[P];
  const double dg = i < m ? reg[row] : 1.0;       // padded rows: identity
#pragma unroll
  for (int j = 0; j < P; ++j) {
    double acc = 0.0;
    if (j < m) {                         // wave-uniform; only acc is live across the branch
      double c0 = 0.0, c1 = 0.0;
#pragma unroll
      for (int k = 0; k < KC; k += 2) {
        const double2 yj = *reinterpret_cast<const double2*>(yb + j * WB_LD + q * KC + k);
        c0 = fma(yi[k], yj.x, c0);
        c1 = fma(yi[k + 1], yj.y, c1);
      }
      acc = c0 + c1;
#pragma unroll
      for (int o = P; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
    }
    a[j] = acc + (j == i ? dg : 0.0);
    __builtin_amdgcn_sched_barrier(0);   // one column at a time (unfenced, every column's reads get hoisted)
  }
  double v = i < m ? (double)rating[s + i] : 0.0;
  const int bad = gj_solve<P>(a, v, lane, gbuf[w]);
  // x = Y_u^T a, lane = rank entry
  double x = 0.0;
#pragma unroll
  for (int t = 0; t < P; ++t) x = fma(readlane_f64(v, t), yb[t * WB_LD + lane], x);   // rows t >= m are 0
  if (lane < r) X[row * r + lane] = (float)x;
  if (lane == 0) status[row] = bad | (deg > P);
}

// Push-through solve for explicit rows with 9..16 ratings on the f64 matrix cores (the bulk of the user sweep:
// the LDS-staged version above reads 128 KB of LDS per user for the Gram alone and is LDS-bandwidth bound).
// One wave per row, no LDS:
//   lane (g = lane >> 4, t = lane & 15) loads columns 16g .. 16g+15 of neighbour t (four 16-byte loads);
//   K = Y_u Y_u^T (16 x 16, padded rows identity) = 16 v_mfma_f64_16x16x4 whose A and B operands are the SAME
//   register (A[m][k] = y_m[k], B[k][n] = y_n[k], with the k order permuted per step: the sum is over all k);
//   -K^-1 by the 16-step sweep (sweep_neg_inv16, shared with als_mfma_solve), a = K^-1 r by tvec;
//   x = Y_u^T a as a 16-lane reduce-scatter (4 xor stages, 8 + 4 + 2 + 1 shuffles) that leaves x[lane] on lane.
// fp64 throughout; results equal the LDS version to fp64 rounding.
__global__ __launch_bounds__(64 * MF_WAVES, 3) void als_woodbury16_mfma(const int64_t* __restrict__ indptr,
                                                                      const int32_t* __restrict__ nbr,
                                                                      const float* __restrict__ rating,
                                                                      const float* __restrict__ Y, int r,
                                                                      const double* __restrict__ reg,
                                                                      const int64_t* __restrict__ rows,
                                                                      int64_t nrows, float* __restrict__ X,
                                                                      int32_t* __restrict__ status) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t idx = (int64_t)blockIdx.x * MF_WAVES + w;
  if (idx >= nrows) return;
  const int64_t row = rows[idx];
  const int64_t s = indptr[row];
  const int64_t deg = indptr[row + 1] - s;
  const int m = __builtin_amdgcn_readfirstlane(deg > 16 ? 0 : (int)deg);
  const int g = lane >> 4, t = lane & 15;
  float y[16];
  if (t < m) {
    const float* yr = Y + (int64_t)nbr[s + t] * r;
    if ((r & 3) == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = 16 * g + 4 * c;
        float4 q4 = col < r ? *reinterpret_cast<const float4*>(yr + col) : float4{0.f, 0.f, 0.f, 0.f};
        y[4 * c] = q4.x;
        y[4 * c + 1] = q4.y;
        y[4 * c + 2] = q4.z;
        y[4 * c + 3] = q4.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) y[c] = 16 * g + c < r ? yr[16 * g + c] : 0.f;
    }
  } else {
#pragma unroll
    for (int c = 0; c < 16; ++c) y[c] = 0.f;
  }
  d4_t K = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double yc = (double)y[c];
    K = mf64(yc, yc, K);
  }
  // + reg on the diagonal (padded rows: identity); C-layout: lane holds K[g + 4q][t]
  const double lam = reg[row];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (g + 4 * q == t) K[q] += t < m ? lam : 1.0;
  const double v = lane < m ? (double)rating[s + lane] : 0.0;      // r_u, entry t on lane t
  int bad = 0;
  const d4_t Kn = sweep_neg_inv16(K, lane, bad);
  const double a = -tvec(Kn, v, 0, g);                              // a[t] on every lane with column t
  // x[16 g + c] = sum_t a_t y_t[16 g + c]: reduce-scatter over the 16 lanes of group g
  double p[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) p[c] = a * (double)y[c];
#pragma unroll
  for (int hb = 8; hb >= 1; hb >>= 1) {
    const bool up = (t & hb) != 0;                                  // this lane keeps the upper half
#pragma unroll
    for (int c = 0; c < hb; ++c) {
      const double send = up ? p[c] : p[c + hb];
      const double recv = __shfl_xor(send, hb);
      p[c] = (up ? p[c + hb] : p[c]) + recv;
    }
  }
  if (lane < r) X[row * r + lane] = (float)p[0];
  if (lane == 0) status[row] = bad | (deg > 16);
}

// heavy rows, pass 1: one wave per (row, chunk of `chunk` neighbours) adds its partial Gram / rhs into fp64
// global accumulators G [nh][RP][RP], B [nh][RP] (device-scope atomics; a 1e6-neighbour item is 1e6/chunk waves
// instead of one serial wave)
template <int RP>
__global__ __launch_bounds__(64) void als_heavy_gram(const int64_t* __restrict__ indptr,
                                                     const int32_t* __restrict__ nbr,
                                                     const float* __restrict__ rating, const float* __restrict__ Y,
                                                     int r, int implicit, float alpha,
                                                     const int64_t* __restrict__ rows,
                                                     const int64_t* __restrict__ chunk_row,
                                                     const int64_t* __restrict__ chunk_start, int64_t chunk,
                                                     double* __restrict__ G, double* __restrict__ B) {
  const int lane = threadIdx.x;
  const int64_t h = chunk_row[blockIdx.x];
  const int64_t row = rows[h];
  const int64_t s = chunk_start[blockIdx.x];
  const int64_t e = min(indptr[row + 1], s + chunk);
  double a[RP];
#pragma unroll
  for (int i = 0; i < RP; ++i) a[i] = 0.0;
  double v = 0.0;
  gram_regs<RP>(nbr, rating, Y, r, implicit, alpha, s, e, lane, a, v);
  if (lane < RP) {
#pragma unroll
    for (int i = 0; i < RP; ++i) unsafeAtomicAdd(G + (h * RP + lane) * RP + i, a[i]);
    unsafeAtomicAdd(B + h * RP + lane, v);
  }
}

// heavy rows, pass 1 on MFMA (rank 64): a 256-thread workgroup per (row, chunk) forms the chunk's partial Gram
// G = sum_t c_t y_t y_t^T as Y_c^T Y_c on the bf16 matrix cores without losing fp32 accuracy: every fp32 factor
// value is split exactly into three bf16 pieces y = hi + mid + lo, and the six cross products with magnitude
// >= 2^-16 (hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi) run as v_mfma_f32_16x16x32_bf16 -- each bf16 x bf16
// product is exact in fp32, the dropped terms are <= 2^-23 relative.  The fp32 MFMA accumulator covers one
// 32-neighbour step only and is folded into fp64 registers after it, so accumulation error does not grow with
// the degree.  Workgroup layout: the 32 neighbours' rows are staged in LDS as [piece][dim][k] bf16 (row stride
// 40 elements: the 16 lanes of a ds_read_b128 group hit disjoint banks); wave w owns Gram tile row w (tiles
// (w, 0..3) of 16 x 16).  The rhs sum_t w_t y_t accumulates in LDS fp64.  Partial G / B are added to the global
// fp64 accumulators as before.  (The VALU version: 64 fp64 FMAs per neighbour per lane, one wave per chunk.)
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int kHK = 32;                 // neighbours per MFMA K-step
constexpr int kHS = 40;                 // LDS row stride (bf16 elements) of a [dim][k] piece

__device__ __forceinline__ void split3(float y, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)y;
  const float r1 = y - (float)hi;
  mid = (__bf16)r1;
  lo = (__bf16)(r1 - (float)mid);
}

template <bool IMPL>
__global__ __launch_bounds__(256) void als_heavy_gram_mfma(const int64_t* __restrict__ indptr,
                                                           const int32_t* __restrict__ nbr,
                                                           const float* __restrict__ rating,
                                                           const float* __restrict__ Y, int r, float alpha,
                                                           const int64_t* __restrict__ rows,
                                                           const int64_t* __restrict__ chunk_row,
                                                           const int64_t* __restrict__ chunk_start, int64_t chunk,
                                                           double* __restrict__ G, double* __restrict__ B) {
  // pieces 0..2: B side (y); IMPL adds pieces 3..5: A side (c y)
  constexpr int NP = IMPL ? 6 : 3;
  __shared__ __bf16 sp[NP][64 * kHS];
  __shared__ double srhs[64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t h = chunk_row[blockIdx.x];
  const int64_t row = rows[h];
  const int64_t s = chunk_start[blockIdx.x];
  const int64_t e = min(indptr[row + 1], s + chunk);
  if (tid < 64) srhs[tid] = 0.0;
  double g64[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) g64[j][i] = 0.0;
  const int sk = tid >> 3, sd = (tid & 7) * 8;        // staging: neighbour sk, dims sd .. sd+7
  const int li = lane & 15, kg = (lane >> 4) * 8;
  for (int64_t t0 = s; t0 < e; t0 += kHK) {
    __syncthreads();                                    // previous step's fragments consumed
    {
      const int64_t t = t0 + sk;
      float yv[8];
      float c = 0.f, wr = 0.f;
      if (t < e) {
        const float* yr = Y + (int64_t)nbr[t] * r;
#pragma unroll
        for (int q = 0; q < 8; ++q) yv[q] = sd + q < r ? yr[sd + q] : 0.f;
        const float rt = rating[t];
        if (IMPL) {
          c = rt > 0.f ? alpha * rt : 0.f;
          wr = rt > 0.f ? 1.f + c : 0.f;
        } else {
          c = 1.f;
          wr = rt;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) yv[q] = 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        __bf16 a, b, d;
        split3(yv[q], a, b, d);
        const int o = (sd + q) * kHS + sk;
        sp[0][o] = a;
        sp[1][o] = b;
        sp[2][o] = d;
        if (IMPL) {
          split3(c * yv[q], a, b, d);
          sp[3][o] = a;
          sp[4][o] = b;
          sp[5][o] = d;
        }
        if (wr != 0.f) atomicAdd(&srhs[sd + q], (double)wr * (double)yv[q]);
      }
    }
    __syncthreads();
    constexpr int AO = IMPL ? 3 : 0;
    bf16x8_t a[3];
#pragma unroll
    for (int p = 0; p < 3; ++p)
      a[p] = *reinterpret_cast<const bf16x8_t*>(&sp[AO + p][(16 * w + li) * kHS + kg]);
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      bf16x8_t b[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) b[p] = *reinterpret_cast<const bf16x8_t*>(&sp[p][(16 * J + li) * kHS + kg]);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) g64[J][i] += (double)acc[i];
    }
  }
  __syncthreads();
  // lane l of wave w holds tile (w, J) entries [m = 4 (l >> 4) + i][n = l & 15]
#pragma unroll
  for (int J = 0; J < 4; ++J)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gm = 16 * w + 4 * (lane >> 4) + i, gn = 16 * J + (lane & 15);
      unsafeAtomicAdd(G + (h * 64 + gm) * 64 + gn, g64[J][i]);
    }
  if (tid < 64) unsafeAtomicAdd(B + h * 64 + tid, srhs[tid]);
}

// heavy rows, pass 2: solve from the accumulated G / B
template <int RP>
__global__ __launch_bounds__(64) void als_heavy_solve(const double* __restrict__ G, const double* __restrict__ B,
                                                      int r, const double* __restrict__ reg,
                                                      const double* __restrict__ YtY,
                                                      const int64_t* __restrict__ rows, float* __restrict__ X,
                                                      int32_t* __restrict__ status) {
  const int lane = threadIdx.x;
  const int64_t h = blockIdx.x;
  const int64_t row = rows[h];
  double a[RP];
#pragma unroll
  for (int i = 0; i < RP; ++i) a[i] = lane < RP ? G[(h * RP + lane) * RP + i] : 0.0;
  double v = lane < RP ? B[h * RP + lane] : 0.0;
  add_reg<RP>(a, lane, r, reg[row], YtY);
  const int bad = chol_solve_regs<RP>(a, v, lane);
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
// rows (nullable): the nrows row ids to solve (light rows); null -> rows 0..nrows-1.
int alink_als_fused_solve(const int64_t* indptr, const int32_t* nbr, const float* rating, const float* Y,
                          int64_t nrows, int r, int implicit, float alpha, const double* reg, const double* YtY,
                          const int64_t* rows, float* X, int32_t* status, hipStream_t stream) {
  if (nrows <= 0) return 0;
  if (r <= 0 || r > 64) return 1;
  const dim3 grid((unsigned)((nrows + GJ_WAVES - 1) / GJ_WAVES)), block(64 * GJ_WAVES);
#define ALS_LAUNCH(RP) hipLaunchKernelGGL(als_fused_solve<RP>, grid, block, 0, stream, indptr, nbr, rating, Y, r, \
                                          implicit, alpha, reg, YtY, rows, nrows, X, status)
  if (r <= 8) ALS_LAUNCH(8);
  else if (r <= 16) ALS_LAUNCH(16);
  else if (r <= 32) ALS_LAUNCH(32);
  else ALS_LAUNCH(64);
#undef ALS_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Heavy rows (degree >> chunk): nh rows, nchunks (row, start) work items; G [nh][RP][RP] and B [nh][RP] must be
// zeroed, RP = the padded rank (8/16/32/64, see alink_als_padded_rank).
int alink_als_heavy_solve(const int64_t* indptr, const int32_t* nbr, const float* rating, const float* Y, int r,
                          int implicit, float alpha, const double* reg, const double* YtY, const int64_t* rows,
                          int64_t nh, const int64_t* chunk_row, const int64_t* chunk_start, int64_t nchunks,
                          int64_t chunk, double* G, double* B, float* X, int32_t* status, int heavy_mfma,
                          hipStream_t stream) {
  if (nh <= 0) return 0;
  if (r <= 0 || r > 64 || nchunks <= 0 || chunk <= 0) return 1;
#define ALS_HEAVY(RP)                                                                                          \
  hipLaunchKernelGGL(als_heavy_gram<RP>, dim3((unsigned)nchunks), dim3(64), 0, stream, indptr, nbr, rating, Y, r, \
                     implicit, alpha, rows, chunk_row, chunk_start, chunk, G, B);                              \
  hipLaunchKernelGGL(als_heavy_solve<RP>, dim3((unsigned)nh), dim3(64), 0, stream, G, B, r, reg, YtY, rows, X, status)
  if (r <= 8) { ALS_HEAVY(8); }
  else if (r <= 16) { ALS_HEAVY(16); }
  else if (r <= 32) { ALS_HEAVY(32); }
  else if (heavy_mfma) {
    // rank 33..64: partial Grams on the matrix cores (exact bf16 x3 split), then the same solve
    if (implicit)
      hipLaunchKernelGGL(als_heavy_gram_mfma<true>, dim3((unsigned)nchunks), dim3(256), 0, stream, indptr, nbr, rating,
                         Y, r, alpha, rows, chunk_row, chunk_start, chunk, G, B);
    else
      hipLaunchKernelGGL(als_heavy_gram_mfma<false>, dim3((unsigned)nchunks), dim3(256), 0, stream, indptr, nbr,
                         rating, Y, r, alpha, rows, chunk_row, chunk_start, chunk, G, B);
    hipLaunchKernelGGL(als_heavy_solve<64>, dim3((unsigned)nh), dim3(64), 0, stream, G, B, r, reg, YtY, rows, X,
                       status);
  } else { ALS_HEAVY(64); }
#undef ALS_HEAVY
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Explicit rows with at most P (8, 16 or 32) neighbours, P < padded rank: the m x m push-through solve above.
int alink_als_woodbury_solve(const int64_t* indptr, const int32_t* nbr, const float* rating, const float* Y,
                             int64_t nrows, int r, const double* reg, const int64_t* rows, int P, float* X,
                             int32_t* status, hipStream_t stream) {
  if (nrows <= 0) return 0;
  if (r <= 0 || r > 64 || rows == nullptr) return 1;
  const dim3 grid((unsigned)((nrows + WB_WAVES - 1) / WB_WAVES)), block(64 * WB_WAVES);
  if (P == 8)
    hipLaunchKernelGGL(als_woodbury_solve<8>, grid, block, 0, stream, indptr, nbr, rating, Y, r, reg, rows, nrows,
                       X, status);
  else if (P == 16)
    hipLaunchKernelGGL(als_woodbury_solve<16>, grid, block, 0, stream, indptr, nbr, rating, Y, r, reg, rows, nrows,
                       X, status);
  else if (P == 32)
    hipLaunchKernelGGL(als_woodbury_solve<32>, grid, block, 0, stream, indptr, nbr, rating, Y, r, reg, rows, nrows,
                       X, status);
  else
    return 1;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Light rows of rank 33..64 on the matrix cores (als_mfma_solve): same contract as alink_als_fused_solve.
int alink_als_mfma_solve(const int64_t* indptr, const int32_t* nbr, const float* rating, const float* Y,
                         int64_t nrows, int r, int implicit, float alpha, const double* reg, const double* YtY,
                         const int64_t* rows, float* X, int32_t* status, hipStream_t stream) {
  if (nrows <= 0) return 0;
  if (r <= 32 || r > 64) return 1;
  const dim3 grid((unsigned)((nrows + MF_WAVES - 1) / MF_WAVES)), block(64 * MF_WAVES);
#define ALS_MF(V, I) hipLaunchKernelGGL((als_mfma_solve<V, I>), grid, block, 0, stream, indptr, nbr, rating, Y, r, \
                                        alpha, reg, YtY, rows, nrows, X, status)
  const bool v4 = r % 4 == 0;
  if (v4 && implicit) ALS_MF(true, true);
  else if (v4) ALS_MF(true, false);
  else if (implicit) ALS_MF(false, true);
  else ALS_MF(false, false);
#undef ALS_MF
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Explicit rows with <= 16 ratings on the matrix cores (als_woodbury16_mfma); same contract as
// alink_als_woodbury_solve with P = 16.
int alink_als_woodbury16_mfma(const int64_t* indptr, const int32_t* nbr, const float* rating, const float* Y,
                              int64_t nrows, int r, const double* reg, const int64_t* rows, float* X, int32_t* status,
                              hipStream_t stream) {
  if (nrows <= 0) return 0;
  if (r <= 0 || r > 64 || rows == nullptr) return 1;
  hipLaunchKernelGGL(als_woodbury16_mfma, dim3((unsigned)((nrows + MF_WAVES - 1) / MF_WAVES)), dim3(64 * MF_WAVES), 0,
                     stream, indptr, nbr, rating, Y, r, reg, rows, nrows, X, status);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int alink_als_padded_rank(int r) { return r <= 8 ? 8 : r <= 16 ? 16 : r <= 32 ? 32 : 64; }

}  // extern "C"
