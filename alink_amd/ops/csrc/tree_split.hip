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

constexpr int QR = 128;   // rows per quantize tile
constexpr int QF = 16;    // features per quantize tile (16 x 256 fp64 thresholds = 32 KiB LDS)

template <typename T>
__device__ __forceinline__ double ldv(const void* p, int64_t i) {
    return (double)reinterpret_cast<const T*>(p)[i];
}

__global__ __launch_bounds__(256) void tree_quantize_kernel(const int64_t* __restrict__ col_ptr,
                                                           const int64_t* __restrict__ null_ptr,
                                                           const int32_t* __restrict__ col_is_f32,
                                                           const int32_t* __restrict__ out_col, int Fc, int64_t n,
                                                           int F, const double* __restrict__ thr,
                                                           const int32_t* __restrict__ nthr, int T, int missing,
                                                           uint8_t* __restrict__ out) {
    extern __shared__ double sthr[];                       // [QF][T]
    __shared__ uint8_t tile[QR][QF];
    const int f0 = blockIdx.y * QF;
    const int fg = min(QF, Fc - f0);
    for (int i = threadIdx.x; i < fg * T; i += 256) sthr[i] = thr[(int64_t)f0 * T + i];
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * QR;
    // lane -> (row, feature): consecutive lanes take consecutive rows of one feature (coalesced column reads)
    for (int e = threadIdx.x; e < QR * QF; e += 256) {
        const int f = e / QR, rl = e - f * QR;
        const int64_t r = r0 + rl;
        if (f >= fg || r >= n) continue;
        const int c = f0 + f;
        const double x = col_is_f32[c] ? ldv<float>((const void*)col_ptr[c], r) : ldv<double>((const void*)col_ptr[c], r);
        const uint8_t* nm = reinterpret_cast<const uint8_t*>(null_ptr[c]);
        int b;
        if (x != x || (nm != nullptr && nm[r])) {
            b = missing;
        } else {
            int lo = 0, hi = nthr[c];
            const double* t = sthr + f * T;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (t[mid] < x) lo = mid + 1;
                else hi = mid;
            }
            b = lo;
        }
        tile[rl][f] = (uint8_t)b;
    }
    __syncthreads();
    // write back: rows of fg bytes at out[r][out_col[f0 + f]]; contiguous when the output columns are
    for (int e = threadIdx.x; e < QR * QF; e += 256) {
        const int rl = e / QF, f = e - rl * QF;
        const int64_t r = r0 + rl;
        if (f < fg && r < n) out[r * F + out_col[f0 + f]] = tile[rl][f];
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

}  // namespace

extern "C" {

// Quantize Fc continuous columns into the uint8 [n, F] bin matrix.  col_ptr/null_ptr/col_is_f32/out_col are
// DEVICE arrays [Fc] (null_ptr entries may be 0); thr [Fc][T] fp64 (padded), nthr [Fc].
int alink_tree_quantize(const int64_t* col_ptr, const int64_t* null_ptr, const int32_t* col_is_f32,
                        const int32_t* out_col, int Fc, int64_t n, int F, const double* thr, const int32_t* nthr,
                        int T, int missing, uint8_t* out, void* stream) {
    if (n <= 0 || Fc <= 0) return 0;
    if (T < 1 || T > 256 || missing < 0 || missing > 255) return 1;
    const dim3 grid((unsigned)((n + QR - 1) / QR), (unsigned)((Fc + QF - 1) / QF));
    hipLaunchKernelGGL(tree_quantize_kernel, grid, dim3(256), (size_t)QF * T * sizeof(double),
                       reinterpret_cast<hipStream_t>(stream), col_ptr, null_ptr, col_is_f32, out_col, Fc, n, F, thr,
                       nthr, T, missing, out);
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
