// Tree preprocessing and split search on CDNA4 (gfx950 / MI355X): kernels K5 and K8 of SURVEY §2.13.
//
// K5 quantize (reference Preprocessing.java quantile discretizer + DataFormatToArray.java:77-83): continuous
//   feature columns (separate fp32/fp64 device arrays, the MTable layout) -> the row-major uint8 bin matrix the
//   histogram kernel reads.  One workgroup per (128-row x 16-feature) tile: the tile's fp64 thresholds sit in
//   LDS (16 x T), every lane binary-searches its values there (bin = #thresholds < x, NaN / null -> missing
//   bin, = torch.searchsorted(thr, x, right=False)), the uint8 tile is transposed through LDS and written as
//   16-byte row segments.  Replaces F strided torch.searchsorted passes over column views of the bin matrix.
//
// K8 GBDT split search (reference CalBestSplit.java:51-218): one 64-lane wave per (node, feature).  Bins
//   0..B-2 (B-1 is the missing bin) are split 4 per lane; the (g, h, count) prefix sums come from a lane-local
//   scan plus a wave exclusive scan (__shfl_up, fp64), the candidate gain |GL^2/HL + GR^2/HR - G^2/H| is
//   masked by the same admissibility rules as the vectorised torch search (hessian ratio, minSamplesPerLeaf,
//   minSumHessianPerLeaf), and the first maximum over bins is reduced across the wave.  Output per (node,
//   feature): best gain (-inf if none) and its bin; the host picks the best feature per node.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr int QR = 128;    // rows per quantize tile
constexpr int QF = 16;     // features per quantize tile (16 x 256 fp64 thresholds = 32 KiB LDS)
constexpr int QRB = 4096;  // rows per workgroup: the thresholds are staged once per 4096 rows, not per tile

template <typename T>
__device__ __forceinline__ double ldv(const void* p, int64_t i) {
    return (double)reinterpret_cast<const T*>(p)[i];
}

// K5 quantize: bin = #thresholds < x (lower bound; NaN / null -> missing), row-major uint8 output.  A workgroup
// owns QF features x QRB rows: it stages the features' thresholds in LDS once (padded to TP = a power of two
// with +inf), then walks its rows in 128-row tiles; every thread bins 8 (row, feature) elements per tile with
// a BRANCHLESS binary search, the 8 searches interleaved (ILP instead of 8 dependent LDS-latency chains), and
// the tile goes out as 16-byte row pieces.
__global__ __launch_bounds__(256) void tree_quantize_kernel(const int64_t* __restrict__ col_ptr,
                                                           const int64_t* __restrict__ null_ptr,
                                                           const int32_t* __restrict__ col_is_f32,
                                                           const int32_t* __restrict__ out_col, int Fc, int64_t n,
                                                           int F, const double* __restrict__ thr, int T, int TP,
                                                           int missing, uint8_t* __restrict__ out) {
    extern __shared__ double sthr[];                       // [QF][TP]
    __shared__ uint8_t tile[QR][QF];
    const int f0 = blockIdx.y * QF;
    const int fg = min(QF, Fc - f0);
    for (int i = threadIdx.x; i < QF * TP; i += 256) {
        const int f = i / TP, j = i - f * TP;
        sthr[i] = (f < fg && j < T) ? thr[(int64_t)(f0 + f) * T + j] : __builtin_inf();
    }
    __syncthreads();
    const int rl = threadIdx.x & (QR - 1);
    const int fsub = threadIdx.x >> 7;                     // 0 / 1: this thread's features are fsub + 2 i
    const void* cp[8];
    const uint8_t* np[8];
    bool f32[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int c = f0 + min(fsub + 2 * i, fg - 1);
        cp[i] = (const void*)col_ptr[c];
        np[i] = reinterpret_cast<const uint8_t*>(null_ptr[c]);
        f32[i] = col_is_f32[c] != 0;
    }
    const int64_t rb0 = (int64_t)blockIdx.x * QRB;
    const int64_t rb1 = rb0 + QRB < n ? rb0 + QRB : n;
    for (int64_t r0 = rb0; r0 < rb1; r0 += QR) {
        const int64_t r = r0 + rl;
        const bool rok = r < rb1;
        double x[8];
        int pos[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            x[i] = rok ? (f32[i] ? ldv<float>(cp[i], r) : ldv<double>(cp[i], r)) : 0.0;
            pos[i] = 0;
        }
        for (int step = TP >> 1; step >= 1; step >>= 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                pos[i] += sthr[(fsub + 2 * i) * TP + pos[i] + step - 1] < x[i] ? step : 0;
        }
        if (TP == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) pos[i] = sthr[(fsub + 2 * i) * TP] < x[i] ? 1 : 0;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = fsub + 2 * i;
            const bool miss = x[i] != x[i] || (rok && np[i] != nullptr && np[i][r]);
            if (f < fg) tile[rl][f] = (uint8_t)(miss ? missing : pos[i]);
        }
        __syncthreads();
        for (int e = threadIdx.x; e < QR * QF; e += 256) {
            const int tr = e / QF, f = e - tr * QF;
            const int64_t rr = r0 + tr;
            if (f < fg && rr < rb1) out[rr * F + out_col[f0 + f]] = tile[tr][f];
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void gbdt_split_kernel(const float* __restrict__ H, int m, int F, int B, int S,
                                                        int gi, int hi, int ci, double min_leaf,
                                                        double min_hess, double* __restrict__ best_gain,
                                                        int32_t* __restrict__ best_bin) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= (int64_t)m * F) return;
    const float* h = H + wave * (int64_t)B * S;          // [B][S] of this (node, feature)
    const int nb = B - 1;                                 // candidate bins (missing bin excluded)
    // lane-local bins 4*lane .. 4*lane+3
    double g[4], hh[4], c[4];
    double sg = 0.0, sh = 0.0, sc = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int b = 4 * lane + k;
        const bool in = b < nb;
        sg += in ? (double)h[b * S + gi] : 0.0;
        sh += in ? (double)h[b * S + hi] : 0.0;
        sc += in ? (double)h[b * S + ci] : 0.0;
        g[k] = sg;
        hh[k] = sh;
        c[k] = sc;
    }
    // wave exclusive scan of the lane totals
    double eg = sg, eh = sh, ec = sc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double tg = __shfl_up(eg, o), th = __shfl_up(eh, o), tc = __shfl_up(ec, o);
        if (lane >= o) {
            eg += tg;
            eh += th;
            ec += tc;
        }
    }
    eg -= sg;
    eh -= sh;
    ec -= sc;
    // node totals = all candidate bins + the missing bin
    const double Gv = __shfl(eg + sg, 63), Hv = __shfl(eh + sh, 63), Cv = __shfl(ec + sc, 63);
    const double G = Gv + (double)h[nb * S + gi], Ht = Hv + (double)h[nb * S + hi], Ct = Cv + (double)h[nb * S + ci];
    const double sH = Ht == 0.0 ? 1.0 : Ht;
    const double base = G * G / sH;
    double bestv = -INFINITY;
    int bestb = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int b = 4 * lane + k;
        if (b >= nb) continue;
        const double GL = eg + g[k], HL = eh + hh[k], CL = ec + c[k];
        const double GR = G - GL, HR = Ht - HL;
        double gain = 0.0;
        if (HL != 0.0 && HR != 0.0) gain = fabs(GL * GL / HL + GR * GR / HR - base);
        const double ratio = HL / (Ht < 1e-6 ? 1.0 : Ht);
        const bool ok = Ht >= 1e-6 && ratio >= 1e-7 && ratio <= 1.0 - 1e-7 && CL >= min_leaf &&
                        Ct - CL >= min_leaf && HL >= min_hess && HR >= min_hess;
        const double v = ok ? gain : -INFINITY;
        if (v > bestv) {          // strict: keeps the first (lowest) bin of this lane on ties
            bestv = v;
            bestb = b;
        }
    }
    // first maximum across the wave: larger gain wins, equal gains -> lower bin
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(bestv, o);
        const int ob = __shfl_xor(bestb, o);
        if (ov > bestv || (ov == bestv && ob < bestb)) {
            bestv = ov;
            bestb = ob;
        }
    }
    if (lane == 0) {
        best_gain[wave] = bestv;
        best_bin[wave] = bestb == 0x7fffffff ? 0 : bestb;
    }
}

// K8/K10 general split search (reference CalBestSplit.java:98-218 for GBDT incl. categorical bins ordered by
// g/h, seriestree/CategoricalSplitter + ContinuousSplitter + Criteria.java for RF / decision trees: Gini,
// information gain, gain ratio, MSE).  One 64-lane wave per (node, feature):
//   1. categorical features: every candidate bin's ordering key (GBDT g/h, MSE mean, classification class-0
//      share; empty bins last) goes to LDS and each bin's rank in the stable order (key, bin) is counted
//      against all bins -> perm[rank] = bin (continuous features keep the identity order);
//   2. the S statistics of the bins in that order: lane-local sums of 4 positions, a wave exclusive scan per
//      statistic, then a sequential walk over the lane's 4 positions gives the left statistics L at every
//      candidate, R = T - L;
//   3. the criterion's gain with the same admissibility rules as the vectorised torch search, and the first
//      maximum over positions.  Output per (node, feature): best gain (-inf if none) and its position j in the
//      sorted order (left child = perm[0..j]).
constexpr int kMaxS = 33;
enum Crit { C_GBDT = 0, C_GINI = 1, C_INFO = 2, C_RATIO = 3, C_MSE = 4 };

__device__ __forceinline__ double lg2(double p) { return p > 0.0 ? log(p) * 1.4426950408889634 : 0.0; }

template <int S>
struct Imp {
  // weight and impurity of a statistics vector (engine._weight / engine._impurity)
  __device__ static double weight(const double* x, int crit, int ncls) {
    if (crit == C_GBDT) return x[2];
    if (crit == C_MSE) return x[0];
    double w = 0.0;
    for (int k = 0; k < ncls; ++k) w += x[k];
    return w;
  }
  __device__ static double impurity(const double* x, int crit, int ncls) {
    const double w = weight(x, crit, ncls);
    if (w < 1e-15) return 0.0;
    if (crit == C_MSE) {
      const double mean = x[1] / w;
      return x[2] / w - mean * mean;
    }
    double acc = 0.0;
    for (int k = 0; k < ncls; ++k) {
      const double p = x[k] / w;
      acc += crit == C_GINI ? p * p : p * lg2(p);
    }
    return crit == C_GINI ? 1.0 - acc : -acc;
  }
};

template <int S>
__global__ __launch_bounds__(256) void tree_split_kernel(const float* __restrict__ H, int m, int F, int B, int crit,
                                                        int ncls, const uint8_t* __restrict__ is_cat,
                                                        double min_leaf, double min_hess, double min_ratio,
                                                        double min_gain, double* __restrict__ best_gain,
                                                        int32_t* __restrict__ best_pos) {
  __shared__ double skey[4][256];
  __shared__ int sperm[4][256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wv;
  if (wave >= (int64_t)m * F) return;                  // whole wave: no block barrier below
  const int f = (int)(wave % F);
  const float* h = H + wave * (int64_t)B * S;          // [B][S]
  const int nb = B - 1;
  const bool cat = is_cat[f] != 0;
  // ---- 1. order
  if (cat) {
    for (int b = lane; b < nb; b += 64) {
      const float* x = h + b * S;
      double key;
      if (crit == C_GBDT) {
        const double g = x[1], hh = x[2];
        key = hh < 1e-6 ? -1.0 : g / hh;
      } else {
        // MSE: mean label; classification: share of class 0 (engine._search); empty bins sort last
        const double cnt = x[S - 1];
        double ww = 0.0;
        if (crit == C_MSE) ww = x[0];
        else
          for (int k = 0; k < ncls; ++k) ww += x[k];
        const double num = crit == C_MSE ? (double)x[1] : (double)x[0];
        key = cnt > 0.0 ? num / (ww == 0.0 ? 1.0 : ww) : INFINITY;
      }
      skey[wv][b] = key;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);                  // lgkmcnt(0): this wave's LDS stores landed
    for (int b = lane; b < nb; b += 64) {
      const double kb = skey[wv][b];
      int rank = 0;
      for (int c = 0; c < nb; ++c) {
        const double kc = skey[wv][c];
        rank += (kc < kb || (kc == kb && c < b)) ? 1 : 0;
      }
      sperm[wv][rank] = b;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
  // ---- 2. prefix statistics in sorted order
  double lsum[S];
#pragma unroll
  for (int k = 0; k < S; ++k) lsum[k] = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int pos = 4 * lane + q;
    if (pos < nb) {
      const int b = cat ? sperm[wv][pos] : pos;
#pragma unroll
      for (int k = 0; k < S; ++k) lsum[k] += (double)h[b * S + k];
    }
  }
  double off[S], tot[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    double e = lsum[k];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double t = __shfl_up(e, o);
      if (lane >= o) e += t;
    }
    tot[k] = __shfl(e, 63);                               // all candidate bins (missing excluded)
    off[k] = e - lsum[k];
  }
  double miss[S];
#pragma unroll
  for (int k = 0; k < S; ++k) miss[k] = (double)h[nb * S + k];
  // totals the gain is taken against: GBDT includes the missing bin (it goes right), the others do not
  double T[S];
#pragma unroll
  for (int k = 0; k < S; ++k) T[k] = crit == C_GBDT ? tot[k] + miss[k] : tot[k];
  const double wT = Imp<S>::weight(T, crit, ncls);
  const double impT = crit == C_GBDT ? 0.0 : Imp<S>::impurity(T, crit, ncls);
  const double cM = miss[S - 1];
  // ---- 3. walk the lane's positions
  double bestv = -INFINITY;
  int bestp = 0x7fffffff;
  double L[S];
#pragma unroll
  for (int k = 0; k < S; ++k) L[k] = off[k];
  for (int q = 0; q < 4; ++q) {
    const int pos = 4 * lane + q;
    if (pos >= nb) break;
    const int b = cat ? sperm[wv][pos] : pos;
    const double cb = (double)h[b * S + (S - 1)];
#pragma unroll
    for (int k = 0; k < S; ++k) L[k] += (double)h[b * S + k];
    double R[S];
#pragma unroll
    for (int k = 0; k < S; ++k) R[k] = T[k] - L[k];
    double gain;
    bool ok;
    if (crit == C_GBDT) {
      const double G = T[1], Ht = T[2], GL = L[1], HL = L[2], GR = G - GL, HR = Ht - HL;
      gain = (HL != 0.0 && HR != 0.0)
                 ? fabs(GL * GL / HL + GR * GR / HR - G * G / (Ht == 0.0 ? 1.0 : Ht)) : 0.0;
      const double ratio = HL / (Ht < 1e-6 ? 1.0 : Ht);
      const double cT = T[S - 1], cL = L[S - 1];
      ok = Ht >= 1e-6 && ratio >= 1e-7 && ratio <= 1.0 - 1e-7 && cL >= min_leaf && cT - cL >= min_leaf &&
           HL >= min_hess && HR >= min_hess;
    } else {
      const double safe = wT < 1e-15 ? 1.0 : wT;
      const double pl = Imp<S>::weight(L, crit, ncls) / safe, pr = Imp<S>::weight(R, crit, ncls) / safe;
      gain = impT - pl * Imp<S>::impurity(L, crit, ncls) - pr * Imp<S>::impurity(R, crit, ncls);
      if (crit == C_RATIO) {
        const double iv = -(pl * lg2(pl) + pr * lg2(pr));
        gain = iv < 1e-15 ? 0.0 : gain / iv;
      }
      if (wT < 1e-15) gain = 0.0;
      const double cL = L[S - 1], cR = R[S - 1], cT = cL + cR;
      const double den = cT + cM == 0.0 ? 1.0 : cT + cM;
      ok = cL > 0.0 && cR > 0.0 && min_leaf <= cL + cM && min_leaf <= cR + cM && min_ratio <= (cL + cM) / den &&
           min_ratio <= (cR + cM) / den && (!cat || cb > 0.0) && gain > 0.0 && gain >= min_gain;
    }
    const double v = ok ? gain : -INFINITY;
    if (v > bestv) {
      bestv = v;
      bestp = pos;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bestv, o);
    const int op = __shfl_xor(bestp, o);
    if (ov > bestv || (ov == bestv && op < bestp)) {
      bestv = ov;
      bestp = op;
    }
  }
  if (lane == 0) {
    best_gain[wave] = bestv;
    best_pos[wave] = bestp == 0x7fffffff ? 0 : bestp;
  }
}

template <int S>
void launch_split(dim3 grid, hipStream_t st, const float* H, int m, int F, int B, int crit, int ncls,
                  const uint8_t* is_cat, double a, double b, double c, double d, double* g, int32_t* p) {
  hipLaunchKernelGGL(tree_split_kernel<S>, grid, dim3(256), 0, st, H, m, F, B, crit, ncls, is_cat, a, b, c, d, g, p);
}


// K5 for fp32 columns with fp32 thresholds: u[j] = the smallest float strictly greater than the fp64 threshold
// t[j] (NaN for the +inf padding), so for any fp32 x: t[j] < x  <=>  u[j] <= x, and the bin count
// #{t < x} is exact while the LDS table and every search read are half the size of the fp64 kernel's.  A
// workgroup owns QF2 = 32 features x QRB rows; a tile is 64 rows x 32 features (thread = row t & 63, features
// (t >> 6) + 4 i, i < 8: a wave reads 64 consecutive rows of one column per load).  Each tile row goes out as
// four 8-byte stores when the group's 32 destination columns are contiguous and 8-byte aligned (F % 8 == 0),
// otherwise byte by byte.
constexpr int QF2 = 32;
constexpr int QR2 = 64;

__global__ __launch_bounds__(256) void tree_quantize_f32_kernel(const int64_t* __restrict__ col_ptr,
                                                               const int64_t* __restrict__ null_ptr,
                                                               const int32_t* __restrict__ out_col, int Fc,
                                                               int64_t n, int F, const float* __restrict__ thr,
                                                               int TP, int missing, uint8_t* __restrict__ out) {
    extern __shared__ float sthr32[];                      // [QF2][TP]
    __shared__ uint8_t tile[QR2][QF2];
    const int f0 = blockIdx.y * QF2;
    const int fg = min(QF2, Fc - f0);
    for (int i = threadIdx.x; i < QF2 * TP; i += 256) {
        const int f = i / TP;
        sthr32[i] = f < fg ? thr[(int64_t)(f0 + f) * TP + (i - f * TP)] : __builtin_nanf("");
    }
    // 8-byte row pieces: the group's destinations are out_col[f0] .. out_col[f0] + 31 and 8-aligned
    bool vec = fg == QF2 && (F & 7) == 0 && (out_col[f0] & 7) == 0;
    for (int f = 1; vec && f < QF2; ++f) vec = out_col[f0 + f] == out_col[f0] + f;
    __syncthreads();
    const int rl = threadIdx.x & (QR2 - 1);
    const int fsub = threadIdx.x >> 6;
    const float* cp[8];
    const uint8_t* np[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int c = f0 + min(fsub + 4 * i, fg - 1);
        cp[i] = reinterpret_cast<const float*>(col_ptr[c]);
        np[i] = reinterpret_cast<const uint8_t*>(null_ptr[c]);
    }
    const int64_t rb0 = (int64_t)blockIdx.x * QRB;
    const int64_t rb1 = rb0 + QRB < n ? rb0 + QRB : n;
    for (int64_t r0 = rb0; r0 < rb1; r0 += QR2) {
        const int64_t r = r0 + rl;
        const bool rok = r < rb1;
        float x[8];
        int pos[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            x[i] = rok ? cp[i][r] : 0.0f;
            pos[i] = 0;
        }
        for (int step = TP >> 1; step >= 1; step >>= 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                pos[i] += sthr32[(fsub + 4 * i) * TP + pos[i] + step - 1] <= x[i] ? step : 0;
        }
        if (TP == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) pos[i] = sthr32[(fsub + 4 * i) * TP] <= x[i] ? 1 : 0;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = fsub + 4 * i;
            const bool miss = x[i] != x[i] || (rok && np[i] != nullptr && np[i][r]);
            if (f < fg) tile[rl][f] = (uint8_t)(miss ? missing : pos[i]);
        }
        __syncthreads();
        if (vec) {
            const int tr = threadIdx.x >> 2, q = threadIdx.x & 3;       // 64 rows x 4 pieces of 8 bytes
            const int64_t rr = r0 + tr;
            if (rr < rb1)
                *reinterpret_cast<uint64_t*>(out + rr * F + out_col[f0] + 8 * q) =
                    *reinterpret_cast<const uint64_t*>(&tile[tr][8 * q]);
        } else {
            for (int e = threadIdx.x; e < QR2 * QF2; e += 256) {
                const int tr = e / QF2, f = e - tr * QF2;
                const int64_t rr = r0 + tr;
                if (f < fg && rr < rb1) out[rr * F + out_col[f0 + f]] = tile[tr][f];
            }
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" {

// Quantize Fc continuous columns into the uint8 [n, F] bin matrix.  col_ptr/null_ptr/col_is_f32/out_col are
// DEVICE arrays [Fc] (null_ptr entries may be 0); thr [Fc][T] fp64 (padded), nthr [Fc].
int alink_tree_quantize(const int64_t* col_ptr, const int64_t* null_ptr, const int32_t* col_is_f32,
                        const int32_t* out_col, int Fc, int64_t n, int F, const double* thr, const int32_t* nthr,
                        int T, int missing, uint8_t* out, void* stream) {
    if (n <= 0 || Fc <= 0) return 0;
    if (T < 1 || T > 256 || missing < 0 || missing > 255) return 1;
    (void)nthr;                           // padded with +inf past each column's count: the search needs no count
    int TP = 1;
    while (TP < T) TP <<= 1;
    const dim3 grid((unsigned)((n + QRB - 1) / QRB), (unsigned)((Fc + QF - 1) / QF));
    hipLaunchKernelGGL(tree_quantize_kernel, grid, dim3(256), (size_t)QF * TP * sizeof(double),
                       reinterpret_cast<hipStream_t>(stream), col_ptr, null_ptr, col_is_f32, out_col, Fc, n, F, thr,
                       T, TP, missing, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// fp32 columns, fp32 "smallest float above the threshold" tables [Fc][TP] (TP a power of two <= 256, NaN pad)
int alink_tree_quantize_f32(const int64_t* col_ptr, const int64_t* null_ptr, const int32_t* out_col, int Fc,
                            int64_t n, int F, const float* thr, int TP, int missing, uint8_t* out, void* stream) {
    if (n <= 0 || Fc <= 0) return 0;
    if (TP < 1 || TP > 256 || (TP & (TP - 1)) != 0 || missing < 0 || missing > 255) return 1;
    const dim3 grid((unsigned)((n + QRB - 1) / QRB), (unsigned)((Fc + QF2 - 1) / QF2));
    hipLaunchKernelGGL(tree_quantize_f32_kernel, grid, dim3(256), (size_t)QF2 * TP * sizeof(float),
                       reinterpret_cast<hipStream_t>(stream), col_ptr, null_ptr, out_col, Fc, n, F, thr, TP, missing,
                       out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Best GBDT split bin per (node, feature) from the fp32 histogram H [m][F][B][S] (stat columns gi, hi, ci).
int alink_gbdt_split(const float* H, int m, int F, int B, int S, int gi, int hi, int ci, double min_leaf,
                     double min_hess, double* best_gain, int32_t* best_bin, void* stream) {
    if (m <= 0 || F <= 0) return 0;
    if (B < 2 || B > 257) return 1;
    const int64_t waves = (int64_t)m * F;
    hipLaunchKernelGGL(gbdt_split_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), H, m, F, B, S, gi, hi, ci, min_leaf, min_hess, best_gain,
                       best_bin);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"

extern "C" {

// General best-split search (categorical + continuous, GBDT / Gini / InfoGain / InfoGainRatio / MSE) over the
// fp32 histogram H [m][F][B][S]; is_cat [F] uint8 (device).  S must be one of the instantiated sizes.
int alink_tree_split(const float* H, int m, int F, int B, int S, int crit, int ncls, const uint8_t* is_cat,
                     double min_leaf, double min_hess, double min_ratio, double min_gain, double* best_gain,
                     int32_t* best_pos, void* stream) {
    if (m <= 0 || F <= 0) return 0;
    if (B < 2 || B > 257 || crit < 0 || crit > 4) return 1;
    if (crit == C_GBDT && S != 4 && S != 3) return 1;
    const int64_t waves = (int64_t)m * F;
    const dim3 grid((unsigned)((waves + 3) / 4));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (S) {
        case 3: launch_split<3>(grid, st, H, m, F, B, crit, ncls, is_cat, min_leaf, min_hess, min_ratio, min_gain, best_gain, best_pos); break;
        case 4: launch_split<4>(grid, st, H, m, F, B, crit, ncls, is_cat, min_leaf, min_hess, min_ratio, min_gain, best_gain, best_pos); break;
        case 5: launch_split<5>(grid, st, H, m, F, B, crit, ncls, is_cat, min_leaf, min_hess, min_ratio, min_gain, best_gain, best_pos); break;
        case 6: launch_split<6>(grid, st, H, m, F, B, crit, ncls, is_cat, min_leaf, min_hess, min_ratio, min_gain, best_gain, best_pos); break;
        case 8: launch_split<8>(grid, st, H, m, F, B, crit, ncls, is_cat, min_leaf, min_hess, min_ratio, min_gain, best_gain, best_pos); break;
        case 11: launch_split<11>(grid, st, H, m, F, B, crit, ncls, is_cat, min_leaf, min_hess, min_ratio, min_gain, best_gain, best_pos); break;
        default: return 3;   // caller falls back to the torch search
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
