// GBDT learning-to-rank gradients (K6, segmented per query) on CDNA4 (gfx950 / MI355X).
//
// Reference: A/operator/common/tree/parallelcart/ConstructLocalBin.java:296-460 (algoType 2 = LambdaMART-NDCG,
// 3 = LambdaMART-DCG, 4 = GBRank), rows of one query contiguous (InitialTrainningBuffer.java:157-235), gains
// label' = 2^min(label, 31) - 1 stored as float, predictions float, gradient / Hessian accumulated in float.
//
// The reference walks every ordered pair (i1, i2) of a query and, when label[i2] < label[i1], adds the pair's
// lambda to g[i1], subtracts it from g[i2] and adds the pair Hessian to both — each add rounding the float
// accumulator.  Element m therefore receives, in this order: its "low" contributions from i1 = 0..m-1, its "high"
// contributions over i2 = 0..n-1, then its "low" contributions from i1 = m+1..n-1.  Here one thread owns one row
// and replays exactly that sequence, so there is no atomic and no reordering: the result is the reference's,
// up to the last-ulp behaviour of exp.
//
//   * one 64-thread workgroup per query (queries are short; a long query loops its rows over the wave);
//   * prediction ranks and label ranks are the reference's stable descending sorts (Arrays.sort of Integer
//     indices with FloatIndexGtComparator), computed as counts: rank(m) = #{p_j > p_m} + #{j < m : p_j == p_m};
//   * inverse max DCG = 1 / sum_r disc[r] * label_sorted_desc[r], summed sequentially in rank order (float
//     products, double sum) like the reference; disc[] is the reference's float table log 2 / log(2 + r),
//     passed in from the host so CPU and GPU use the same values;
//   * output: the {g*g, g, h, 1} row records the histogram kernels consume (weights applied as for the other
//     losses), after the reference's |g| < 1e-7 or |h| < 1e-7 -> (0, 0) rule.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int RK_T = 64;

__device__ __forceinline__ void pair_terms(int algo, float ph, float pl, float yh, float yl, float dh, float dl,
                                           bool spread, double inv_max_dcg, double& lam, double& hes, bool& skip) {
    const float dsf = ph - pl;                  // float - float, widened (Java: double deltaScore = highPred - lowPred)
    const double ds = (double)dsf;
    if (algo == 4) {
        skip = ds >= 0.6;
        lam = 0.0;
        hes = 1.0;
        return;
    }
    skip = false;
    double dn = ((double)yh - (double)yl) * (double)fabsf(dh - dl);
    if (yh != yl && spread) dn /= ((double)0.01f + fabs(ds));
    if (algo == 2) dn *= inv_max_dcg;
    double l = 2.0 / (1.0 + exp(2.0 * ds));
    double h = l * (2.0 - l);
    lam = l * -dn;
    hes = h * (2.0 * dn);
}

__global__ __launch_bounds__(RK_T) void gbdt_rank_stats_kernel(const float* __restrict__ pred,
                                                               const float* __restrict__ lab,
                                                               const float* __restrict__ w,
                                                               const int64_t* __restrict__ off, int ngroups,
                                                               const float* __restrict__ disc, int algo,
                                                               int* __restrict__ rank_scratch,
                                                               float* __restrict__ sorted_scratch,
                                                               float4* __restrict__ stats) {
    const int gi = blockIdx.x;
    if (gi >= ngroups) return;
    const int tid = threadIdx.x;
    const int64_t b = off[gi];
    const int n = (int)(off[gi + 1] - b);
    if (n <= 0) return;          // an empty query has no pairs (uniform over the block: before any barrier)
    const float* P = pred + b;
    const float* Y = lab + b;
    int* R = rank_scratch + b;
    float* S = sorted_scratch + b;
    __shared__ double inv_sh;
    __shared__ int spread_sh;
    for (int m = tid; m < n; m += RK_T) {
        const float pm = P[m], ym = Y[m];
        int rp = 0, rl = 0;
        for (int j = 0; j < n; ++j) {
            const float pj = P[j], yj = Y[j];
            rp += (pj > pm) || (pj == pm && j < m);
            rl += (yj > ym) || (yj == ym && j < m);
        }
        R[m] = rp;
        S[rl] = ym;
    }
    __syncthreads();
    if (tid == 0) {
        double md = 0.0;
        float best = P[0], worst = P[0];
        for (int r = 0; r < n; ++r) {
            md += (double)(disc[r] * S[r]);
            best = P[r] > best ? P[r] : best;
            worst = P[r] < worst ? P[r] : worst;
        }
        inv_sh = 1.0 / md;
        spread_sh = best != worst;
    }
    __syncthreads();
    const double inv = inv_sh;
    const bool spread = spread_sh != 0;
    for (int m = tid; m < n; m += RK_T) {
        const float pm = P[m], ym = Y[m], dm = disc[R[m]];
        float g = 0.f, h = 0.f;
        double lam, hes;
        bool skip;
        for (int j = 0; j < n; ++j) {
            if (j == m) {
                // m as the higher-labelled row of every pair (m, i2)
                for (int i2 = 0; i2 < n; ++i2) {
                    if (i2 == m || !(Y[i2] < ym)) continue;
                    pair_terms(algo, pm, P[i2], ym, Y[i2], dm, disc[R[i2]], spread, inv, lam, hes, skip);
                    if (skip) continue;
                    if (algo == 4) lam = -((double)P[i2] + 0.6);
                    g = (float)((double)g + lam);
                    h = (float)((double)h + hes);
                }
            } else if (ym < Y[j]) {
                // m as the lower-labelled row of the pair (j, m)
                pair_terms(algo, P[j], pm, Y[j], ym, disc[R[j]], dm, spread, inv, lam, hes, skip);
                if (skip) continue;
                if (algo == 4) g = (float)((double)g + -((double)P[j] - 0.6));
                else g = (float)((double)g - lam);
                h = (float)((double)h + hes);
            }
        }
        if (((double)g < 1e-7 && (double)g > -1e-7) || ((double)h < 1e-7 && (double)h > -1e-7)) {
            g = 0.f;
            h = 0.f;
        }
        if (w != nullptr) {
            const float ww = w[b + m];
            g *= ww;
            h *= ww;
        }
        stats[b + m] = make_float4(g * g, g, h, 1.0f);
    }
}

}  // namespace

extern "C" {

// {g*g, g, h, 1} ranking row records for ngroups contiguous queries (rows off[q] .. off[q+1]-1, each <= 10000
// rows: the reference's kMaxPosition); rank_scratch (int [N]) and sorted_scratch (float [N]) are work space
int alink_gbdt_rank_stats(const void* pred, const void* lab, const void* w, const int64_t* off, int ngroups,
                          const void* disc, int algo, void* rank_scratch, void* sorted_scratch, void* stats,
                          void* stream) {
    if (ngroups <= 0) return 0;
    if (algo < 2 || algo > 4) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(gbdt_rank_stats_kernel, dim3(ngroups), dim3(RK_T), 0, (hipStream_t)stream, (const float*)pred,
                       (const float*)lab, (const float*)w, off, ngroups, (const float*)disc, algo, (int*)rank_scratch,
                       (float*)sorted_scratch, (float4*)stats);
    return (int)hipGetLastError();
}

}  // extern "C"
