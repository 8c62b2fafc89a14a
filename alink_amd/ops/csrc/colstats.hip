// One-pass column statistics of a dense row-major matrix — gfx950 / MI355X.
//
// Reference: DenseVectorSummarizer.visit (A/common/statistics/basicstatistic/DenseVectorSummarizer.java:78-120)
// walks every vector and updates sum, squareSum, normL1, min, max and numNonZero per dimension; the summaries of
// the partitions are merged on one task (StatisticsHelper.summary).  Here one launch reads the matrix once in its
// native dtype (no fp64 staging copy):
//
//   * workgroup (256 threads) = one row slab x one chunk of <= 256 columns; when d < 256 the workgroup holds
//     P = 256 / d row phases, thread (phase, c) reads X[row0 + phase + P*i][c] so consecutive threads touch
//     consecutive addresses of the same rows (fully coalesced);
//   * fp64 accumulators for sum / sum^2 / |x|, exact min / max, integer non-zero counts, in registers;
//   * phases are folded through LDS in fixed phase order and each workgroup writes one [6][chunk] partial;
//     the host sums the [slabs][6][d] partials in slab order -> bit-reproducible for a given shape.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int TB = 256;

template <typename T>
__device__ __forceinline__ double to_d(T v) { return (double)v; }
template <>
__device__ __forceinline__ double to_d<__bf16>(__bf16 v) { return (double)(float)v; }

// NaN-propagating min / max (java.lang.Math.min / torch.min semantics, unlike fmin)
__device__ __forceinline__ double nmin(double a, double b) { return (b < a || b != b) ? b : a; }
__device__ __forceinline__ double nmax(double a, double b) { return (b > a || b != b) ? b : a; }

template <typename T>
__global__ __launch_bounds__(TB) void colstats_kernel(const T* __restrict__ X, int64_t n, int d, int64_t rows_per,
                                                      double* __restrict__ part) {
    __shared__ double red[TB];
    const int tid = threadIdx.x;
    const int c0 = blockIdx.y * TB;
    const int dc = d - c0 < TB ? d - c0 : TB;               // columns of this chunk
    const int P = TB / dc;                                  // row phases
    const int ph = tid / dc, c = tid % dc;
    const bool act = ph < P;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per;
    const int64_t r1 = r0 + rows_per < n ? r0 + rows_per : n;
    // 4 independent accumulator sets (4 rows in flight per thread), combined in fixed order below
    double s4[4] = {0.0, 0.0, 0.0, 0.0}, q4[4] = {0.0, 0.0, 0.0, 0.0}, a4[4] = {0.0, 0.0, 0.0, 0.0};
    double lo4[4], hi4[4], z4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < 4; ++u) { lo4[u] = __builtin_inf(); hi4[u] = -__builtin_inf(); }
    if (act) {
        const T* p = X + (int64_t)c0 + c;
        int64_t r = r0 + ph;
        for (; r + 3 * (int64_t)P < r1; r += 4 * (int64_t)P) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = to_d(p[(r + u * (int64_t)P) * d]);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s4[u] += v[u];
                q4[u] += v[u] * v[u];
                a4[u] += fabs(v[u]);
                lo4[u] = nmin(lo4[u], v[u]);
                hi4[u] = nmax(hi4[u], v[u]);
                z4[u] += v[u] != 0.0 ? 1.0 : 0.0;
            }
        }
        for (int u = 0; r < r1; r += P, ++u) {
            const double v = to_d(p[r * d]);
            s4[u] += v;
            q4[u] += v * v;
            a4[u] += fabs(v);
            lo4[u] = nmin(lo4[u], v);
            hi4[u] = nmax(hi4[u], v);
            z4[u] += v != 0.0 ? 1.0 : 0.0;
        }
    }
    const double s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    const double s2 = (q4[0] + q4[1]) + (q4[2] + q4[3]);
    const double l1 = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    const double mn = nmin(nmin(lo4[0], lo4[1]), nmin(lo4[2], lo4[3]));
    const double mx = nmax(nmax(hi4[0], hi4[1]), nmax(hi4[2], hi4[3]));
    const double nz = (z4[0] + z4[1]) + (z4[2] + z4[3]);
    // fold phases in fixed order: sums through LDS, then min / max
    double* out = part + (int64_t)blockIdx.x * 6 * d + c0;
    double vals[6] = {s, s2, l1, mn, mx, nz};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        red[tid] = vals[k];
        __syncthreads();
        if (tid < dc) {
            double a = red[tid];
            for (int q = 1; q < P; ++q) {
                const double b = red[tid + q * dc];
                a = k == 3 ? nmin(a, b) : k == 4 ? nmax(a, b) : a + b;
            }
            out[(int64_t)k * d + tid] = a;
        }
        __syncthreads();
    }
}

template <typename T>
int launch(const void* X, int64_t n, int d, int slabs, double* part, void* stream) {
    const int64_t rows_per = (n + slabs - 1) / slabs;
    const dim3 grid((unsigned)slabs, (unsigned)((d + TB - 1) / TB));
    hipLaunchKernelGGL(colstats_kernel<T>, grid, dim3(TB), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const T*>(X), n, d, rows_per, part);
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// part: [slabs][6][d] fp64 = (sum, sum of squares, sum |x|, min, max, non-zero count) of each row slab.
// dtype: 0 fp32, 1 fp64, 2 bf16.
int alink_colstats(const void* X, int64_t n, int d, int dtype, int slabs, double* part, void* stream) {
    if (n < 0 || d <= 0 || slabs <= 0) return -1;
    switch (dtype) {
        case 0: return launch<float>(X, n, d, slabs, part, stream);
        case 1: return launch<double>(X, n, d, slabs, part, stream);
        case 2: return launch<__bf16>(X, n, d, slabs, part, stream);
        default: return -2;
    }
}

}  // extern "C"
