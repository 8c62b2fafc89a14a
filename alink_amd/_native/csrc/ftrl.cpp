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

}  // extern "C"
