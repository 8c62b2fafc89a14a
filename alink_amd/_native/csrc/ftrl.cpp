// FTRL-proximal, one sample at a time (reference FtrlTrainStreamOp.CalcTask.flatMap1/flatMap2,
// FtrlTrainStreamOp.java:396-485): margin w.x, p = sigmoid(margin), then per touched coordinate
//   g = (p - y) x_i * scale;  sigma = (sqrt(n_i + g^2) - sqrt(n_i)) / alpha
//   z_i += g - sigma w_i;     n_i += g^2
//   w_i = |z_i| <= l1 ? 0 : (sign(z_i) l1 - z_i) / (beta + sqrt(n_i)/alpha + l2)
// Samples of a micro-batch arrive as CSR (the intercept is column 0 when present); the update is strictly
// sequential, so it runs on the host core that owns the stream partition.
#include <cmath>
#include <cstdint>

extern "C" {

int alink_ftrl_update_csr(const int64_t* indptr, const int32_t* indices, const double* values, const double* label,
                          int64_t nrows, double* w, double* n, double* z, int64_t dim, double alpha, double beta,
                          double l1, double l2, double scale) {
  for (int64_t r = 0; r < nrows; ++r) {
    const int64_t s = indptr[r], e = indptr[r + 1];
    double wx = 0.0;
    for (int64_t k = s; k < e; ++k) {
      const int32_t i = indices[k];
      if (i < 0 || i >= dim) return 1;
      wx += values[k] * w[i];
    }
    const double p = 1.0 / (1.0 + std::exp(-wx));
    for (int64_t k = s; k < e; ++k) {
      const int32_t i = indices[k];
      const double g = (p - label[r]) * values[k] * scale;
      const double sigma = (std::sqrt(n[i] + g * g) - std::sqrt(n[i])) / alpha;
      z[i] += g - sigma * w[i];
      n[i] += g * g;
      if (std::fabs(z[i]) <= l1) {
        w[i] = 0.0;
      } else {
        w[i] = ((z[i] < 0 ? -1.0 : 1.0) * l1 - z[i]) / (beta + std::sqrt(n[i]) / alpha + l2);
      }
    }
  }
  return 0;
}

// Feature-sharded micro-batch FTRL (updateMode SHARDED): partial margins of every row on the owned coordinate
// range [lo, hi) (w is the shard, indexed i - lo) ...
int alink_ftrl_partial_margin(const int64_t* indptr, const int32_t* indices, const double* values, int64_t nrows,
                              const double* w, int64_t lo, int64_t hi, double* margin) {
  for (int64_t r = 0; r < nrows; ++r) {
    double wx = 0.0;
    for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k) {
      const int64_t i = indices[k];
      if (i >= lo && i < hi) wx += values[k] * w[i - lo];
    }
    margin[r] = wx;
  }
  return 0;
}

// ... then the owned coordinates replay their entries in sample order with err[r] = sigmoid(margin_r) - y_r
// (the all-reduced margins); same per-coordinate order as the GPU kernel, so both give identical bits up to libm.
int alink_ftrl_shard_update(const int64_t* indptr, const int32_t* indices, const double* values, const double* err,
                            int64_t nrows, double* w, double* n, double* z, int64_t lo, int64_t hi, double alpha,
                            double beta, double l1, double l2) {
  for (int64_t r = 0; r < nrows; ++r) {
    for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k) {
      const int64_t i = (int64_t)indices[k] - lo;
      if (i < 0 || i >= hi - lo) continue;
      // same arithmetic as the GPU replay (ops/csrc/ftrl.hip ftrl_coord_update_kernel)
      const double ia = 1.0 / alpha;
      const double g = err[r] * values[k];
      const double nn = n[i] + g * g;
      const double sn = std::sqrt(nn);
      const double sigma = (sn - std::sqrt(n[i])) * ia;
      const double rden = 1.0 / (beta + sn * ia + l2);
      z[i] += g - sigma * w[i];
      n[i] = nn;
      w[i] = std::fabs(z[i]) <= l1 ? 0.0 : (std::copysign(l1, z[i]) - z[i]) * rden;
    }
  }
  return 0;
}

}  // extern "C"
