// Factorization-machine micro-batch kernels — gfx950 / MI355X, fp64.
//
// Reference: FmOptimizer.UpdateLocalModel.updateFactors (A/operator/common/optim/FmOptimizer.java:389-437) —
// per sample: y = b + <w,x> + 1/2 sum_f ((sum_i v_if x_i)^2 - sum_i v_if^2 x_i^2) (calcY), dL/dy, then AdaGrad on
// the bias, every touched v_i (grad = dldy * x_i * (vx_f - v_if x_i) + lambda2 v_if) and w_i.  On the GPU a
// micro-batch takes its gradient at one model (models/recommendation/fm.py), in two launches:
//
//   fm_forward:       one wave per CSR row, lane f = factor f (k <= 64): vx_f, sum v^2 x^2 and <w,x> over the
//                     row's entries, y by a wave reduction.  Also the batch / stream predictor for sparse rows.
//   fm_coord_update:  entries sorted by coordinate on the device (stable -> sample order inside a coordinate);
//                     one wave per coordinate segment, lane f accumulates the factor gradient and its square in
//                     fp64 over the segment, then applies AdaGrad to v_i, w_i and their sigma in place.  Exactly
//                     one writer per coordinate: no atomics, deterministic, and only touched coordinates are
//                     read or written (the torch path rewrites the whole [D, k] model per micro-batch).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__global__ __launch_bounds__(256) void fm_forward_kernel(const int64_t* __restrict__ indptr,
                                                         const int* __restrict__ idx, const double* __restrict__ val,
                                                         int64_t nrows, int k, const double* __restrict__ w,
                                                         const double* __restrict__ V, double bias,
                                                         double* __restrict__ y, double* __restrict__ vx_out) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = wid; r < nrows; r += nw) {
        const int64_t s = indptr[r], e = indptr[r + 1];
        double vx = 0.0, v2 = 0.0, lin = 0.0;
        for (int64_t p = s; p < e; ++p) {
            const int c = idx[p];
            const double x = val[p];
            if (lane < k) {
                const double v = V[(int64_t)c * k + lane];
                vx += x * v;
                v2 += x * x * v * v;
            }
        }
        if (w != nullptr)
            for (int64_t p = s + lane; p < e; p += 64) lin += val[p] * w[idx[p]];
        const double inter = lane < k ? vx * vx - v2 : 0.0;
        const double tot = wave_sum(lin) + 0.5 * wave_sum(inter);
        if (lane == 0) y[r] = bias + tot;
        if (vx_out != nullptr && lane < k) vx_out[r * k + lane] = vx;
    }
}

__global__ __launch_bounds__(256) void fm_coord_update_kernel(
        const int64_t* __restrict__ seg, int64_t nseg, const int64_t* __restrict__ coord,
        const int64_t* __restrict__ ent_row, const double* __restrict__ ent_val, const double* __restrict__ g,
        const double* __restrict__ vx, const double* __restrict__ sw, int k, double* __restrict__ w,
        double* __restrict__ sg_w, double* __restrict__ V, double* __restrict__ sg_V, double* __restrict__ use,
        double lr, double lam1, double lam2, double eps) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t sgi = wid; sgi < nseg; sgi += nw) {
        const int64_t c = coord[sgi];
        const int64_t a = seg[sgi], b = seg[sgi + 1];
        const double vc = lane < k ? V[c * k + lane] : 0.0;
        const double wc = w != nullptr ? w[c] : 0.0;
        double G = 0.0, S = 0.0, Gl = 0.0, Sl = 0.0, us = 0.0;
        for (int64_t p = a; p < b; ++p) {
            const int64_t r = ent_row[p];
            const double x = ent_val[p];
            const double gr = g[r];
            if (lane < k) {
                const double gv = gr * x * (vx[r * k + lane] - x * vc) + lam2 * vc;
                G += gv;
                S += gv * gv;
            }
            const double gl = gr * x + lam1 * wc;
            Gl += gl;
            Sl += gl * gl;
            us += sw[r];
        }
        if (lane < k) {
            const int64_t o = c * k + lane;
            const double sg = sg_V[o] + S;
            sg_V[o] = sg;
            V[o] = vc - lr * G / sqrt(sg + eps);
        }
        if (lane == 0) {
            if (w != nullptr) {
                const double sg = sg_w[c] + Sl;
                sg_w[c] = sg;
                w[c] = wc - lr * Gl / sqrt(sg + eps);
            }
            use[c] += us;
        }
    }
}

int grid_for(int64_t waves) {
    int64_t g = (waves + 3) / 4;
    return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

extern "C" {

// y[r] = bias + <w, x_r> + 1/2 sum_f (vx_f^2 - sum_i v_if^2 x_i^2); vx_out (nullable) [nrows][k]; w nullable.
int alink_fm_forward_f64(const int64_t* indptr, const int* idx, const double* val, int64_t nrows, int k,
                         const double* w, const double* V, double bias, double* y, double* vx_out, void* stream) {
    if (nrows <= 0) return 0;
    if (k < 0 || k > 64) return -1;
    hipLaunchKernelGGL(fm_forward_kernel, dim3(grid_for(nrows)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       indptr, idx, val, nrows, k, w, V, bias, y, vx_out);
    return (int)hipGetLastError();
}

// AdaGrad on the touched coordinates: entries (ent_row, ent_val) sorted by coordinate, seg[nseg+1] segment
// bounds, coord[nseg] their coordinates; g[row] = dL/dy; w / sg_w nullable (no linear term).
int alink_fm_coord_update_f64(const int64_t* seg, int64_t nseg, const int64_t* coord, const int64_t* ent_row,
                              const double* ent_val, const double* g, const double* vx, const double* sw, int k,
                              double* w, double* sg_w, double* V, double* sg_V, double* use, double lr, double lam1,
                              double lam2, double eps, void* stream) {
    if (nseg <= 0) return 0;
    if (k < 1 || k > 64) return -1;
    hipLaunchKernelGGL(fm_coord_update_kernel, dim3(grid_for(nseg)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), seg, nseg, coord, ent_row, ent_val, g, vx, sw, k, w,
                       sg_w, V, sg_V, use, lr, lam1, lam2, eps);
    return (int)hipGetLastError();
}

}  // extern "C"
