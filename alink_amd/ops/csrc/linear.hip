// Fused one-pass gradient of a linear model's unary loss on CDNA4 (gfx950 / MI355X).
//
// Replaces the reference's per-sample loop UnaryLossObjFunc.updateGradient (UnaryLossObjFunc.java:62-67,
// called from OptimObjFunc.calcGradient, OptimObjFunc.java:126-152) and the two-GEMV torch form
// (eta = X w; grad = X^T (w_i * l'(eta_i, y_i))) with ONE read of X:
//
//   lane-per-row: a lane loads its row x (D_PAD doubles, kept in registers), eta = x . coef,
//   g = weight * l'(eta, y) (the same cut-offs as the reference's loss functions), then acc += g * x and
//   lsum += weight * l(eta, y).  Rows are grid-strided; at the end every block reduces its 256 lane
//   accumulators (wave shuffles + LDS) into one fp64 slab row, and a second kernel sums the slabs in a fixed
//   order (run-to-run deterministic), writing [grad_0..grad_{d-1}, lossSum, weightSum].
//
// Dense fp64 (the reference trains in double): d <= 32 lane-per-row (below), 32 < d <= 1024 lanes-over-columns
// (linear_grad_wide_kernel: 1.54 -> see profiles/linear_grad_wide_r2.txt at d = 64).  Loss codes:
//   0 log (LR)  1 logistic (log / ln2)  2 square  3 hinge  4 smooth hinge  5 perceptron  6 exponential
//   7 huber(param = delta)  8 svr(param = epsilon)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr int THREADS = 256;

__device__ __forceinline__ void loss_and_deriv(int code, double eta, double y, double prm, double& l, double& g) {
    const double d = eta * y;
    switch (code) {
        case 0:
        case 1: {
            const double dc = fmin(fmax(d, -37.0), 34.0);
            if (d < -37.0) {
                l = -d;
                g = -y;
            } else if (d > 34.0) {
                l = 0.0;
                g = 0.0;
            } else {
                l = log1p(exp(-dc));
                g = -y / (exp(dc) + 1.0);
            }
            if (code == 1) {
                const double inv_ln2 = 1.4426950408889634;
                l *= inv_ln2;
                g = (d < -37.0 ? -y : -y / (exp(fmin(d, 700.0)) + 1.0)) * inv_ln2;
            }
            break;
        }
        case 2:
            l = 0.5 * (eta - y) * (eta - y);
            g = eta - y;
            break;
        case 3:
            l = fmax(1.0 - d, 0.0);
            g = d < 1.0 ? -y : 0.0;
            break;
        case 4:
            if (d <= 0.0) {
                l = 0.5 - d;
                g = -y;
            } else if (d >= 1.0) {
                l = 0.0;
                g = 0.0;
            } else {
                l = 0.5 * (1.0 - d) * (1.0 - d);
                g = (1.0 - d) * (-y);
            }
            break;
        case 5:
            l = fmax(-d, 0.0);
            g = d < 0.0 ? -y : 0.0;
            break;
        case 6: {
            const double e = exp(-d);
            l = e;
            g = -y * e;
            break;
        }
        case 7: {
            const double x = eta - y, ax = fabs(x);
            l = ax > prm ? prm * (ax - prm / 2) : x * x / 2;
            g = ax > prm ? copysign(prm, x) : x;
            break;
        }
        default: {
            const double x = eta - y, ax = fabs(x);
            l = fmax(ax - prm, 0.0);
            g = ax > prm ? (x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0)) : 0.0;
            break;
        }
    }
}

template <int DP>
__global__ __launch_bounds__(THREADS) void linear_grad_kernel(const double* __restrict__ X, const double* __restrict__ y,
                                                             const double* __restrict__ wt,
                                                             const double* __restrict__ coef, int64_t n, int d,
                                                             int code, double prm, double* __restrict__ slab) {
    __shared__ double red[THREADS / 64][DP + 2];
    __shared__ double w[DP];
    for (int c = threadIdx.x; c < DP; c += THREADS) w[c] = c < d ? coef[c] : 0.0;
    __syncthreads();
    double acc[DP];
#pragma unroll
    for (int c = 0; c < DP; ++c) acc[c] = 0.0;
    double lsum = 0.0, wsum = 0.0;
    constexpr bool KEEP_X = DP <= 32;   // DP = 64: re-read the (cache-hot) row instead of holding it
    const int64_t stride = (int64_t)gridDim.x * THREADS;
    for (int64_t r = (int64_t)blockIdx.x * THREADS + threadIdx.x; r < n; r += stride) {
        const double* xr = X + r * d;
        double x[KEEP_X ? DP : 1];
        double eta = 0.0;
#pragma unroll
        for (int c = 0; c < DP; ++c) {
            const double v = c < d ? xr[c] : 0.0;
            if constexpr (KEEP_X) x[c] = v;
            eta = fma(v, w[c], eta);
        }
        const double wi = wt[r];
        double l, g;
        loss_and_deriv(code, eta, y[r], prm, l, g);
        g *= wi;
        lsum = fma(wi, l, lsum);
        wsum += wi;
#pragma unroll
        for (int c = 0; c < DP; ++c) {
            double v;
            if constexpr (KEEP_X) v = x[c];
            else v = c < d ? xr[c] : 0.0;
            acc[c] = fma(g, v, acc[c]);
        }
    }
    // block reduction: wave shuffles, then 4 waves through LDS
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < DP + 2; ++c) {
        double v = c < DP ? acc[c] : (c == DP ? lsum : wsum);
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
        if (lane == 0) red[wave][c] = v;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < DP + 2; c += THREADS) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < THREADS / 64; ++q) v += red[q][c];
        slab[(int64_t)blockIdx.x * (DP + 2) + c] = v;
    }
}

// fixed-order sum of the per-block slabs: out = [grad(d), lossSum, weightSum].  One workgroup per output
// column: thread t sums slabs t, t+256, ... and the 256 partials are combined by a fixed LDS tree, so the
// result is run-to-run deterministic.  (A single-thread-per-column loop over 2048 slabs was latency-bound
// at ~0.75 ms, a third of the whole gradient at d = 32.)
__global__ __launch_bounds__(THREADS) void linear_grad_reduce_kernel(const double* __restrict__ slab, int nblk,
                                                                     int dp, int d, double* __restrict__ out) {
    __shared__ double part[THREADS];
    const int c = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < nblk; b += THREADS) s += slab[(int64_t)b * (dp + 2) + c];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = THREADS / 2; off > 0; off >>= 1) {
        if (threadIdx.x < off) part[threadIdx.x] += part[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (c < d) out[c] = part[0];
        else if (c == dp) out[d] = part[0];
        else if (c == dp + 1) out[d + 1] = part[0];
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Wide rows, 32 < d <= 1024: lanes over COLUMNS (lane l owns columns l + 64j, j < NC), RG rows per wave step.
//   * loads: each row is read as NC fully coalesced 512-B wave loads (no per-lane row strides);
//   * eta of the RG rows by a transposing butterfly: log2(RG) exchange steps halve the live row count while
//     pairing lanes (RG/2 + RG/4 + ... + 1 shuffles), then 6 - log2(RG) plain steps — RG + 5 - log2 RG
//     shuffles for RG rows instead of 6 RG; afterwards lane l holds the eta of row rowof(l);
//   * the loss derivative is evaluated by the 64/RG lanes of each row, g_r broadcast back (RG shuffles),
//     acc[j] += g_r x_r[j] — per-lane column accumulators need no cross-lane reduction at the end.
// Blocks grid-stride over row groups; the block partials go to the same slab layout as the narrow kernel
// ([nblk][DP + 2], DP = 64 NC), so the fixed-order reduce kernel below serves both.
// ---------------------------------------------------------------------------------------------------------------
template <int RG>
__device__ __forceinline__ double eta_butterfly(double (&v)[RG], int lane) {
    // exchange steps: xor 32, 16, ... (one per halving of the live row set)
#pragma unroll
    for (int live = RG, bit = 32; live > 1; live >>= 1, bit >>= 1) {
        const bool hi = (lane & bit) != 0;
#pragma unroll
        for (int i = 0; i < live / 2; ++i) {
            const double keep = hi ? v[i + live / 2] : v[i];
            const double send = hi ? v[i] : v[i + live / 2];
            v[i] = keep + __shfl_xor(send, bit);
        }
    }
    double s = v[0];
    constexpr int LOGRG = RG == 1 ? 0 : RG == 2 ? 1 : RG == 4 ? 2 : 3;
#pragma unroll
    for (int bit = 32 >> LOGRG; bit > 0; bit >>= 1) s += __shfl_xor(s, bit);
    return s;
}

// row (within the group) whose eta lane l holds after eta_butterfly<RG>
template <int RG>
__device__ __forceinline__ int row_of_lane(int lane) {
    int r = 0;
#pragma unroll
    for (int live = RG, bit = 32; live > 1; live >>= 1, bit >>= 1) r = 2 * r + ((lane & bit) ? 1 : 0);
    return r;
}

template <int RG>
__device__ __forceinline__ int lane_of_row(int r) {
    int l = 0;
    // bits of r from the most significant (first exchange step, lane bit 32) down
    constexpr int LOGRG = RG == 1 ? 0 : RG == 2 ? 1 : RG == 4 ? 2 : 3;
#pragma unroll
    for (int s = 0; s < LOGRG; ++s) l |= ((r >> (LOGRG - 1 - s)) & 1) ? (32 >> s) : 0;
    return l;
}

template <int NC, int RG>
__global__ __launch_bounds__(THREADS) void linear_grad_wide_kernel(const double* __restrict__ X,
                                                                  const double* __restrict__ y,
                                                                  const double* __restrict__ wt,
                                                                  const double* __restrict__ coef, int64_t n, int d,
                                                                  int code, double prm, double* __restrict__ slab) {
    constexpr int DP = 64 * NC;
    constexpr int NW = THREADS / 64;
    __shared__ double red[NW][DP + 2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double cf[NC], acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const int c = lane + 64 * j;
        cf[j] = c < d ? coef[c] : 0.0;
        acc[j] = 0.0;
    }
    double lsum = 0.0, wsum = 0.0;
    const int myrow = row_of_lane<RG>(lane);
    const bool row_leader = (lane & ((64 / RG) - 1)) == 0;   // one of the 64/RG lanes holding its row's eta
    const int64_t ngroups = (n + RG - 1) / RG;
    const int64_t gstride = (int64_t)gridDim.x * NW;
    for (int64_t grp = (int64_t)blockIdx.x * NW + wave; grp < ngroups; grp += gstride) {
        const int64_t r0 = grp * RG;
        double x[RG][NC], part[RG];
#pragma unroll
        for (int r = 0; r < RG; ++r) {
            const bool ok = r0 + r < n;
            const double* xr = X + (r0 + r) * d;
            double p = 0.0;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const int c = lane + 64 * j;
                x[r][j] = (ok && c < d) ? xr[c] : 0.0;
                p = fma(x[r][j], cf[j], p);
            }
            part[r] = p;
        }
        const double eta = eta_butterfly<RG>(part, lane);
        const int64_t rr = r0 + myrow;
        double gl = 0.0;
        if (rr < n) {
            const double wi = wt[rr];
            double l, g;
            loss_and_deriv(code, eta, y[rr], prm, l, g);
            gl = g * wi;
            if (row_leader) {
                lsum = fma(wi, l, lsum);
                wsum += wi;
            }
        }
#pragma unroll
        for (int r = 0; r < RG; ++r) {
            const double gr = __shfl(gl, lane_of_row<RG>(r));
#pragma unroll
            for (int j = 0; j < NC; ++j) acc[j] = fma(gr, x[r][j], acc[j]);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        lsum += __shfl_xor(lsum, off);
        wsum += __shfl_xor(wsum, off);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) red[wave][lane + 64 * j] = acc[j];
    if (lane == 0) {
        red[wave][DP] = lsum;
        red[wave][DP + 1] = wsum;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < DP + 2; c += THREADS) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < NW; ++q) v += red[q][c];
        slab[(int64_t)blockIdx.x * (DP + 2) + c] = v;
    }
}

template <int NC, int RG>
int launch_wide(const double* X, const double* y, const double* w, const double* coef, int64_t n, int d,
                       int code, double prm, double* slab, int nblk, double* out, hipStream_t st) {
    hipLaunchKernelGGL((linear_grad_wide_kernel<NC, RG>), dim3(nblk), dim3(THREADS), 0, st, X, y, w, coef, n, d, code,
                       prm, slab);
    hipLaunchKernelGGL(linear_grad_reduce_kernel, dim3(64 * NC + 2), dim3(THREADS), 0, st, slab, nblk, 64 * NC, d,
                       out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---------------------------------------------------------------------------------------------------------------
// K14: losses of the adaptive line search in ONE pass over X (reference CalcLosses / UnaryLossObjFunc
// calcSearchValues, A/operator/common/optim/subfunc/CalcLosses.java:41-65, UnaryLossObjFunc.java:98-139):
//   e0 = x.coef, e1 = x.dir (both margins from the same registers), then for s = 0..S
//   loss_s += w l(e0 - s beta e1, y).  Same lanes-over-columns layout and transposing butterfly as the wide
// gradient kernel (both margins reduced together); per-block partial losses -> fixed-order slab reduction.
// ---------------------------------------------------------------------------------------------------------------
constexpr int MAX_STEPS = 16;

template <int NC, int RG>
__global__ __launch_bounds__(THREADS) void linear_search_kernel(const double* __restrict__ X,
                                                               const double* __restrict__ y,
                                                               const double* __restrict__ wt,
                                                               const double* __restrict__ coef,
                                                               const double* __restrict__ dir, int64_t n, int d,
                                                               int code, double prm, double beta, int nsteps,
                                                               double* __restrict__ slab) {
    constexpr int NW = THREADS / 64;
    __shared__ double red[NW][MAX_STEPS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double cf[NC], dv[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const int c = lane + 64 * j;
        cf[j] = c < d ? coef[c] : 0.0;
        dv[j] = c < d ? dir[c] : 0.0;
    }
    double lacc[MAX_STEPS];
#pragma unroll
    for (int s = 0; s < MAX_STEPS; ++s) lacc[s] = 0.0;
    const int myrow = row_of_lane<RG>(lane);
    const bool row_leader = (lane & ((64 / RG) - 1)) == 0;
    const int64_t ngroups = (n + RG - 1) / RG;
    const int64_t gstride = (int64_t)gridDim.x * NW;
    for (int64_t grp = (int64_t)blockIdx.x * NW + wave; grp < ngroups; grp += gstride) {
        const int64_t r0 = grp * RG;
        double p0[RG], p1[RG];
#pragma unroll
        for (int r = 0; r < RG; ++r) {
            const bool ok = r0 + r < n;
            const double* xr = X + (r0 + r) * d;
            double a = 0.0, b = 0.0;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const int c = lane + 64 * j;
                const double v = (ok && c < d) ? xr[c] : 0.0;
                a = fma(v, cf[j], a);
                b = fma(v, dv[j], b);
            }
            p0[r] = a;
            p1[r] = b;
        }
        const double e0 = eta_butterfly<RG>(p0, lane);
        const double e1 = eta_butterfly<RG>(p1, lane);
        const int64_t rr = r0 + myrow;
        if (rr < n && row_leader) {
            const double wi = wt[rr], yi = y[rr];
#pragma unroll
            for (int s = 0; s < MAX_STEPS; ++s) {
                if (s < nsteps) {
                    double l, g;
                    loss_and_deriv(code, e0 - (double)s * beta * e1, yi, prm, l, g);
                    lacc[s] = fma(wi, l, lacc[s]);
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s < MAX_STEPS; ++s) {
        double v = lacc[s];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) red[wave][s] = v;
    }
    __syncthreads();
    if (threadIdx.x < MAX_STEPS + 2) {
        const int c = threadIdx.x;
        double v = 0.0;
        if (c < MAX_STEPS)
#pragma unroll
            for (int q = 0; q < NW; ++q) v += red[q][c];
        slab[(int64_t)blockIdx.x * (MAX_STEPS + 2) + c] = v;
    }
}

template <int NC, int RG>
int launch_search(const double* X, const double* y, const double* w, const double* coef, const double* dir,
                  int64_t n, int d, int code, double prm, double beta, int nsteps, double* slab, int nblk,
                  double* out, hipStream_t st) {
    hipLaunchKernelGGL((linear_search_kernel<NC, RG>), dim3(nblk), dim3(THREADS), 0, st, X, y, w, coef, dir, n, d,
                       code, prm, beta, nsteps, slab);
    // out[0..nsteps) = per-step loss sums (fixed order over blocks); columns past nsteps are zero
    hipLaunchKernelGGL(linear_grad_reduce_kernel, dim3(MAX_STEPS), dim3(THREADS), 0, st, slab, nblk, MAX_STEPS,
                       MAX_STEPS, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

template <int DP>
int launch(const double* X, const double* y, const double* w, const double* coef, int64_t n, int d, int code,
           double prm, double* slab, int nblk, double* out, hipStream_t st) {
    hipLaunchKernelGGL(linear_grad_kernel<DP>, dim3(nblk), dim3(THREADS), 0, st, X, y, w, coef, n, d, code, prm,
                       slab);
    hipLaunchKernelGGL(linear_grad_reduce_kernel, dim3(DP + 2), dim3(THREADS), 0, st, slab, nblk, DP, d, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}


// ---------------------------------------------------------------------------------------------------------------
// Sparse (CSR) gradient, K12 for hashed / one-hot features (UnaryLossObjFunc.java:62-139 on SparseVector data):
//   pass 1, one wave per row: eta = x . coef (lanes over the row's non-zeros, wave reduction), then lane 0
//           writes g_r = w_r l'(eta_r, y_r) and lw_r = w_r l(eta_r, y_r);
//   pass 2, one wave per column over the CSC copy (built once per dataset): grad_j = sum_r x_rj g_r as a
//           gather + fixed-order wave reduction — no atomics, so hot columns (the intercept, frequent hash
//           buckets) cost a longer gather instead of serialised fp64 atomics, and the result is deterministic.
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void csr_row_deriv_kernel(const int64_t* __restrict__ crow,
                                                               const int32_t* __restrict__ col,
                                                               const double* __restrict__ val,
                                                               const double* __restrict__ y,
                                                               const double* __restrict__ w,
                                                               const double* __restrict__ coef, int64_t n, int code,
                                                               double prm, double* __restrict__ g,
                                                               double* __restrict__ lw) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * (THREADS / 64);
    for (int64_t r = w0; r < n; r += nw) {
        double eta = 0.0;
        for (int64_t k = crow[r] + lane; k < crow[r + 1]; k += 64) eta = fma(val[k], coef[col[k]], eta);
        for (int o = 32; o > 0; o >>= 1) eta += __shfl_xor(eta, o);
        if (lane == 0) {
            double l, d;
            loss_and_deriv(code, eta, y[r], prm, l, d);
            g[r] = w[r] * d;
            lw[r] = w[r] * l;
        }
    }
}

__global__ __launch_bounds__(THREADS) void csc_gather_kernel(const int64_t* __restrict__ cptr,
                                                            const int64_t* __restrict__ crow_of,
                                                            const double* __restrict__ cval,
                                                            const double* __restrict__ g, int64_t d,
                                                            double* __restrict__ grad) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * (THREADS / 64);
    for (int64_t j = w0; j < d; j += nw) {
        double s = 0.0;
        for (int64_t k = cptr[j] + lane; k < cptr[j + 1]; k += 64) s = fma(cval[k], g[crow_of[k]], s);
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) grad[j] = s;
    }
}

}  // namespace

extern "C" {

// slab must hold nblk * (pad(d) + 2) doubles, out d + 2 doubles; pad(d) in {8, 16, 32, 64}
int alink_linear_grad_f64(const double* X, const double* y, const double* w, const double* coef, int64_t n, int d,
                          int code, double prm, double* slab, int nblk, double* out, void* stream) {
    if (n <= 0 || d <= 0 || d > 64 || nblk <= 0 || code < 0 || code > 8) return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (d <= 8) return launch<8>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
    if (d <= 16) return launch<16>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
    if (d <= 32) return launch<32>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
    return launch<64>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
}

// K14 line-search losses: out[s] = sum_i w_i l(x_i.coef - s beta x_i.dir, y_i), s < nsteps <= 16, d <= 1024.
// slab: nblk * 18 doubles, out: 16 doubles.
int alink_linear_search_f64(const double* X, const double* y, const double* w, const double* coef, const double* dir,
                            int64_t n, int d, int code, double prm, double beta, int nsteps, double* slab, int nblk,
                            double* out, void* stream) {
    if (n <= 0 || d <= 0 || d > 1024 || nblk <= 0 || code < 0 || code > 8 || nsteps < 1 || nsteps > MAX_STEPS)
        return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch ((d + 63) / 64) {
        case 1: return launch_search<1, 8>(X, y, w, coef, dir, n, d, code, prm, beta, nsteps, slab, nblk, out, st);
        case 2: return launch_search<2, 8>(X, y, w, coef, dir, n, d, code, prm, beta, nsteps, slab, nblk, out, st);
        case 3: case 4:
            return launch_search<4, 4>(X, y, w, coef, dir, n, d, code, prm, beta, nsteps, slab, nblk, out, st);
        case 5: case 6: case 7: case 8:
            return launch_search<8, 2>(X, y, w, coef, dir, n, d, code, prm, beta, nsteps, slab, nblk, out, st);
        default:
            return launch_search<16, 1>(X, y, w, coef, dir, n, d, code, prm, beta, nsteps, slab, nblk, out, st);
    }
}

int alink_linear_grad_pad(int d) {
    if (d > 64 && d <= 1024) {
        const int nc = (d + 63) / 64;
        return 64 * (nc <= 8 ? nc : nc <= 12 ? 12 : 16);     // the NC instantiated for d (launch switch below)
    }
    return d <= 8 ? 8 : d <= 16 ? 16 : d <= 32 ? 32 : 64;
}

// wide dense rows, 32 < d <= 1024 (slab: nblk * (alink_linear_grad_pad(d) + 2) doubles, out d + 2)
int alink_linear_grad_wide_f64(const double* X, const double* y, const double* w, const double* coef, int64_t n,
                               int d, int code, double prm, double* slab, int nblk, double* out, void* stream) {
    if (n <= 0 || d <= 32 || d > 1024 || nblk <= 0 || code < 0 || code > 8) return 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch ((d + 63) / 64) {
        case 1: return launch_wide<1, 8>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 2: return launch_wide<2, 8>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 3: return launch_wide<3, 8>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 4: return launch_wide<4, 8>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 5: return launch_wide<5, 4>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 6: return launch_wide<6, 4>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 7: return launch_wide<7, 4>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 8: return launch_wide<8, 4>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        case 9: case 10: case 11: case 12:
            return launch_wide<12, 2>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
        default: return launch_wide<16, 2>(X, y, w, coef, n, d, code, prm, slab, nblk, out, st);
    }
}

// CSR pass 1: g [n] = w * l'(x.coef, y), lw [n] = w * l(x.coef, y)
int alink_csr_row_deriv_f64(const int64_t* crow, const int32_t* col, const double* val, const double* y,
                            const double* w, const double* coef, int64_t n, int code, double prm, double* g,
                            double* lw, void* stream) {
    if (n <= 0) return 0;
    const int64_t blocks = (n + 3) / 4;
    hipLaunchKernelGGL(csr_row_deriv_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(THREADS), 0,
                       reinterpret_cast<hipStream_t>(stream), crow, col, val, y, w, coef, n, code, prm, g, lw);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// CSC pass 2: grad [d] = X^T g (cptr [d+1], crow_of / cval [nnz] = the CSC copy)
int alink_csc_gather_f64(const int64_t* cptr, const int64_t* crow_of, const double* cval, const double* g, int64_t d,
                         double* grad, void* stream) {
    if (d <= 0) return 0;
    const int64_t blocks = (d + 3) / 4;
    hipLaunchKernelGGL(csc_gather_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(THREADS), 0,
                       reinterpret_cast<hipStream_t>(stream), cptr, crow_of, cval, g, d, grad);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
