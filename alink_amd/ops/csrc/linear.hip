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
// Dense fp64 (the reference trains in double), d <= 64.  Loss codes:
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

int alink_linear_grad_pad(int d) { return d <= 8 ? 8 : d <= 16 ? 16 : d <= 32 ? 32 : 64; }

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
