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

// Wave-cooperative Gibbs sweep: G lanes (G = power of two >= min(K, 64)) own one token, 64 / G tokens per
// wave.  The group reads the token's document row nd[d][.] and word row nw[w][.] as coalesced G-wide segments,
// forms p_k lane-parallel, reduces the total, then walks the chunks again with a segmented inclusive scan and
// picks the first topic whose cdf reaches u * total by a ballot inside the group.  Tokens are document-major,
// so consecutive groups share the document row in cache.  (The thread-per-token kernel above reads both rows
// one element per lane per step: K serial, uncoalesced loads per token, twice.)
template <int G>
__global__ __launch_bounds__(256) void lda_gibbs_wave_kernel(const int64_t* __restrict__ d_tok,
                                                             const int64_t* __restrict__ w_tok,
                                                             const int64_t* __restrict__ z_in, int64_t T, int K,
                                                             const int* __restrict__ nd, const int* __restrict__ nw,
                                                             const double* __restrict__ nk, double alpha,
                                                             double beta, double vbeta,
                                                             const double* __restrict__ u,
                                                             int64_t* __restrict__ z_out) {
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);                        // lane inside the token's group
  const int grp = lane / G;
  constexpr int per_wave = 64 / G;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t t0 = wave * per_wave; t0 < T; t0 += nwaves * per_wave) {
    const int64_t t = t0 + grp;
    const bool live = t < T;
    const int64_t tt = live ? t : T - 1;
    const int64_t d = d_tok[tt], w = w_tok[tt];
    const int z = (int)z_in[tt];
    const int* ndr = nd + d * K;
    const int* nwr = nw + w * K;
    double tot = 0.0;
    for (int c = 0; c < K; c += G) {
      const int k = c + gl;
      double p = 0.0;
      if (k < K) {
        const double own = k == z ? 1.0 : 0.0;
        p = ((double)ndr[k] - own + alpha) * ((double)nwr[k] - own + beta) / (nk[k] - own + vbeta);
      }
      tot += p;
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) tot += __shfl_xor(tot, o, G);
    const double target = (live ? u[t] : 0.0) * tot;
    double run = 0.0;
    int pick = K - 1;
    bool found = false;
    for (int c = 0; c < K && !found; c += G) {        // uniform across the wave only per group: see ballot
      const int k = c + gl;
      double p = 0.0;
      if (k < K) {
        const double own = k == z ? 1.0 : 0.0;
        p = ((double)ndr[k] - own + alpha) * ((double)nwr[k] - own + beta) / (nk[k] - own + vbeta);
      }
      double cum = p;
#pragma unroll
      for (int o = 1; o < G; o <<= 1) {
        const double v = __shfl_up(cum, o, G);
        if (gl >= o) cum += v;
      }
      cum += run;
      const uint64_t hit = __ballot(k < K && cum >= target);
      const uint64_t mine = G == 64 ? hit : (hit >> (grp * G)) & ((1ull << G) - 1ull);
      if (mine != 0ull) {
        pick = c + (int)__builtin_ctzll(mine);
        found = true;
      }
      run = __shfl(cum, (grp * G) + G - 1);
    }
    if (live && gl == 0) z_out[t] = pick;
  }
}

// Online variational Bayes E-step (reference OnlineCorpusStep.java; Hoffman et al. 2010): one wave per
// document runs ALL its fixed-point iterations in registers -- lane l holds topics l, l + 64, ... of gamma,
// expElogtheta and the accumulator; per token the wave reads the word's exp(E log beta) row coalesced, reduces
// phinorm = sum_k et_k eb_wk across lanes, and accumulates eb_wk * cts / phinorm.  Iterates until the mean
// absolute gamma change is <= tol (the torch loop's per-document rule), then writes gamma, expElogtheta and the
// final per-token phinorm.  Replaces a host-synchronised torch loop of [T, K] gathers per iteration.
__device__ double digamma_d(double x) {
  double r = 0.0;
  while (x < 6.0) {
    r -= 1.0 / x;
    x += 1.0;
  }
  const double f = 1.0 / (x * x);
  return r + log(x) - 0.5 / x -
         f * (1.0 / 12 - f * (1.0 / 120 - f * (1.0 / 252 - f * (1.0 / 240 - f * (1.0 / 132)))));
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int KJ>
__global__ __launch_bounds__(256) void lda_estep_kernel(const int64_t* __restrict__ doc_off,
                                                        const int64_t* __restrict__ word,
                                                        const double* __restrict__ cts, int64_t D, int K,
                                                        const double* __restrict__ eb,
                                                        const double* __restrict__ alpha,
                                                        const double* __restrict__ gamma0, int max_iter, double tol,
                                                        double* __restrict__ gamma_out, double* __restrict__ et_out,
                                                        double* __restrict__ phinorm_out) {
  const int lane = threadIdx.x & 63;
  const int64_t d = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= D) return;
  const int64_t t0 = doc_off[d], t1 = doc_off[d + 1];
  double g[KJ], et[KJ], al[KJ];
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int k = lane + 64 * j;
    g[j] = k < K ? gamma0[d * K + k] : 0.0;
    al[j] = k < K ? alpha[k] : 0.0;
  }
  auto expelog = [&]() {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < KJ; ++j) s += g[j];
    const double dsum = digamma_d(wave_sum(s));
#pragma unroll
    for (int j = 0; j < KJ; ++j) et[j] = lane + 64 * j < K ? exp(digamma_d(g[j]) - dsum) : 0.0;
  };
  for (int it = 0; it < max_iter; ++it) {
    expelog();
    double acc[KJ];
#pragma unroll
    for (int j = 0; j < KJ; ++j) acc[j] = 0.0;
    for (int64_t t = t0; t < t1; ++t) {
      const double* ebr = eb + word[t] * K;
      double e[KJ];
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        const int k = lane + 64 * j;
        e[j] = k < K ? ebr[k] : 0.0;
        s += et[j] * e[j];
      }
      const double scale = cts[t] / (wave_sum(s) + 1e-100);
#pragma unroll
      for (int j = 0; j < KJ; ++j) acc[j] += e[j] * scale;
    }
    double ch = 0.0;
#pragma unroll
    for (int j = 0; j < KJ; ++j) {
      const double nv = lane + 64 * j < K ? al[j] + et[j] * acc[j] : 0.0;
      ch += fabs(nv - g[j]);
      g[j] = nv;
    }
    if (wave_sum(ch) / K <= tol) break;
  }
  expelog();
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int k = lane + 64 * j;
    if (k < K) {
      gamma_out[d * K + k] = g[j];
      et_out[d * K + k] = et[j];
    }
  }
  for (int64_t t = t0; t < t1; ++t) {
    const double* ebr = eb + word[t] * K;
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < KJ; ++j) {
      const int k = lane + 64 * j;
      s += k < K ? et[j] * ebr[k] : 0.0;
    }
    s = wave_sum(s);
    if (lane == 0) phinorm_out[t] = s + 1e-100;
  }
}

}  // namespace

extern "C" {

// variant 0: thread per token; 1: wave-cooperative (G lanes per token)
int alink_lda_gibbs(const int64_t* d_tok, const int64_t* w_tok, const int64_t* z_in, int64_t T, int K, const int* nd,
                    const int* nw, const double* nk, double alpha, double beta, double vbeta, const double* u,
                    int64_t* z_out, int variant, void* stream) {
    if (T <= 0) return 0;
    if (K < 1) return -1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (variant == 0) {
        int64_t g = (T + 255) / 256;
        if (g > 16384) g = 16384;
        hipLaunchKernelGGL(lda_gibbs_kernel, dim3((unsigned)g), dim3(256), 0, st, d_tok, w_tok, z_in, T, K, nd, nw, nk,
                           alpha, beta, vbeta, u, z_out);
        return (int)hipGetLastError();
    }
    // wave-cooperative: G lanes per token
    int G = 1;
    while (G < K && G < 64) G <<= 1;
    const int64_t per_wave = 64 / G;
    int64_t g = (T + per_wave * 4 - 1) / (per_wave * 4);
    if (g > 32768) g = 32768;
    switch (G) {
#define ALINK_GW(GG) \
        case GG: hipLaunchKernelGGL(lda_gibbs_wave_kernel<GG>, dim3((unsigned)g), dim3(256), 0, st, d_tok, w_tok, z_in, \
                                    T, K, nd, nw, nk, alpha, beta, vbeta, u, z_out); break;
        ALINK_GW(1) ALINK_GW(2) ALINK_GW(4) ALINK_GW(8) ALINK_GW(16) ALINK_GW(32) ALINK_GW(64)
#undef ALINK_GW
        default: return -1;
    }
    return (int)hipGetLastError();
}

// Online-VB E-step for D documents (tokens grouped by document: doc_off [D+1]); K <= 256.
int alink_lda_estep(const int64_t* doc_off, const int64_t* word, const double* cts, int64_t D, int K, const double* eb,
                    const double* alpha, const double* gamma0, int max_iter, double tol, double* gamma_out,
                    double* et_out, double* phinorm_out, void* stream) {
    if (D <= 0) return 0;
    if (K < 1 || K > 256) return 1;
    const dim3 grid((unsigned)((D + 3) / 4));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int KJ = (K + 63) / 64;
#define ALINK_ES(J) \
    hipLaunchKernelGGL(lda_estep_kernel<J>, grid, dim3(256), 0, st, doc_off, word, cts, D, K, eb, alpha, gamma0, max_iter, \
                       tol, gamma_out, et_out, phinorm_out)
    if (KJ == 1) ALINK_ES(1);
    else if (KJ == 2) ALINK_ES(2);
    else if (KJ == 3) ALINK_ES(3);
    else ALINK_ES(4);
#undef ALINK_ES
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
