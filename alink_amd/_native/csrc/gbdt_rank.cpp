// Host path of the GBDT learning-to-rank gradients (the CPU twin of ops/csrc/gbdt_rank.hip).
//
// A literal transcription of the reference's pair loop (A/operator/common/tree/parallelcart/ConstructLocalBin.java
// :296-430): per query, a stable descending sort of the labels (inverse max DCG) and of the predictions (ranks),
// then every ordered pair (i1, i2) with label[i2] < label[i1] updates the float accumulators g / h of both rows in
// loop order.  The GPU kernel replays the same per-row sequence one thread per row; the two agree up to the
// last-ulp behaviour of exp.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

extern "C" {

// g_out / h_out: float [N]; off: int64 [ngroups + 1] row offsets of the contiguous queries; disc: float [>= max
// query size] = (float)(log 2 / log(2 + r)); algo 2 (NDCG), 3 (DCG), 4 (GBRank).  Returns 0, or -1 on bad input.
int alink_gbdt_rank_grad_host(const float* pred, const float* lab, const int64_t* off, int64_t ngroups,
                              const float* disc, int algo, float* g_out, float* h_out) {
    if (algo < 2 || algo > 4) return -1;
    std::vector<int> by_label, by_pred, rank;
    for (int64_t q = 0; q < ngroups; ++q) {
        const int64_t b = off[q];
        const int n = (int)(off[q + 1] - b);
        if (n <= 0) continue;
        const float* P = pred + b;
        const float* Y = lab + b;
        float* G = g_out + b;
        float* H = h_out + b;
        by_label.resize(n);
        by_pred.resize(n);
        rank.resize(n);
        std::iota(by_label.begin(), by_label.end(), 0);
        std::iota(by_pred.begin(), by_pred.end(), 0);
        std::stable_sort(by_label.begin(), by_label.end(), [&](int a, int c) { return Y[a] > Y[c]; });
        double max_dcg = 0.0;
        for (int r = 0; r < n; ++r) max_dcg += (double)(disc[r] * Y[by_label[r]]);
        const double inverse_max_dcg = 1.0 / max_dcg;
        std::stable_sort(by_pred.begin(), by_pred.end(), [&](int a, int c) { return P[a] > P[c]; });
        for (int r = 0; r < n; ++r) rank[by_pred[r]] = r;
        const double best = P[by_pred[0]], worst = P[by_pred[n - 1]];
        for (int i = 0; i < n; ++i) {
            G[i] = 0.f;
            H[i] = 0.f;
        }
        for (int i1 = 0; i1 < n; ++i1) {
            const double high_label = Y[i1];
            const float high_pred = P[i1];
            const int high_rank = rank[i1];
            for (int i2 = 0; i2 < n; ++i2) {
                if (i2 == i1) continue;
                const float low_pred = P[i2];
                const double low_label = Y[i2];
                const int low_rank = rank[i2];
                if (low_label >= high_label) continue;
                const double delta_score = (double)(float)(high_pred - low_pred);
                if (algo == 4) {
                    const double tau = 0.6;
                    if (delta_score >= tau) continue;
                    G[i1] = (float)((double)G[i1] + -(low_pred + tau));
                    G[i2] = (float)((double)G[i2] + -(high_pred - tau));
                    H[i1] += 1;
                    H[i2] += 1;
                    continue;
                }
                const double dcg_gap = high_label - low_label;
                const double paired_discount = (double)std::fabs(disc[high_rank] - disc[low_rank]);
                double delta_ndcg = dcg_gap * paired_discount;
                if (high_label != low_label && best != worst) delta_ndcg /= ((double)0.01f + std::fabs(delta_score));
                if (algo == 2) delta_ndcg *= inverse_max_dcg;
                double p_lambda = 2.0 / (1.0 + std::exp(2.0 * delta_score));
                double p_hessian = p_lambda * (2.0 - p_lambda);
                p_lambda *= -delta_ndcg;
                p_hessian *= 2 * delta_ndcg;
                G[i1] = (float)((double)G[i1] + p_lambda);
                G[i2] = (float)((double)G[i2] - p_lambda);
                H[i1] = (float)((double)H[i1] + p_hessian);
                H[i2] = (float)((double)H[i2] + p_hessian);
            }
        }
        for (int i = 0; i < n; ++i) {
            if (((double)G[i] < 1e-7 && (double)G[i] > -1e-7) || ((double)H[i] < 1e-7 && (double)H[i] > -1e-7)) {
                G[i] = 0.f;
                H[i] = 0.f;
            }
        }
    }
    return 0;
}

}  // extern "C"
