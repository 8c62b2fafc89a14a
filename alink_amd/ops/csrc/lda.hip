// Collapsed-Gibbs LDA token sweep — gfx950 / MI355X.
//
// Reference: EmCorpusStep (A/operator/common/clustering/lda/EmCorpusStep.java) resamples every token's topic
// from the word-topic counts of the previous superstep, one Java thread per worker; the counts are then summed
// over workers (AD-LDA).  Here one thread owns one token: it evaluates
//     p_k = (n_dk - [z=k] + alpha) (n_wk - [z=k] + beta) / (n_k - [z=k] + V beta)
// over the K topics twice (total, then the inverse-CDF walk with the caller's uniform u) straight from the
// [D][K] / [V][K] int32 count tables — no [T][K] probability / cumsum matrices in HBM (the torch path
// materialises three of them).  Counts are rebuilt afterwards by integer bincounts + one all-reduce.
// fp64 throughout, so the draw equals the torch formula's for the same u.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__global__ __launch_bounds__(256) void lda_gibbs_kernel(const int64_t* __restrict__ d_tok,
                                                        const int64_t* __restrict__ w_tok,
                                                        const int64_t* __restrict__ z_in, int64_t T, int K,
                                                        const int* __restrict__ nd, const int* __restrict__ nw,
                                                        const double* __restrict__ nk, double alpha, double beta,
                                                        double vbeta, const double* __restrict__ u,
                                                        int64_t* __restrict__ z_out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += stride) {
        const int64_t d = d_tok[t], w = w_tok[t];
        const int z = (int)z_in[t];
        const int* ndr = nd + d * K;
        const int* nwr = nw + w * K;
        double tot = 0.0;
        for (int k = 0; k < K; ++k) {
            const double own = k == z ? 1.0 : 0.0;
            tot += ((double)ndr[k] - own + alpha) * ((double)nwr[k] - own + beta) / (nk[k] - own + vbeta);
        }
        const double target = u[t] * tot;
        double cum = 0.0;
        int pick = K - 1;
        for (int k = 0; k < K; ++k) {
            const double own = k == z ? 1.0 : 0.0;
            cum += ((double)ndr[k] - own + alpha) * ((double)nwr[k] - own + beta) / (nk[k] - own + vbeta);
            if (cum >= target) {            // first k with cdf >= u * total (torch.searchsorted, left side)
                pick = k;
                break;
            }
        }
        z_out[t] = pick;
    }
}

}  // namespace

extern "C" {

int alink_lda_gibbs(const int64_t* d_tok, const int64_t* w_tok, const int64_t* z_in, int64_t T, int K, const int* nd,
                    const int* nw, const double* nk, double alpha, double beta, double vbeta, const double* u,
                    int64_t* z_out, void* stream) {
    if (T <= 0) return 0;
    if (K < 1) return -1;
    int64_t g = (T + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(lda_gibbs_kernel, dim3((unsigned)g), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), d_tok,
                       w_tok, z_in, T, K, nd, nw, nk, alpha, beta, vbeta, u, z_out);
    return (int)hipGetLastError();
}

}  // extern "C"
