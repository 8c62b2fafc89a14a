// f64 MFMA probe (gfx950): (1) the operand / result lane maps of v_mfma_f64_16x16x4f64 checked with exact
// integer data, including an accumulator tile fed back as the next product's B operand (register s = k-step s)
// and as the A operand of its transpose; (2) throughput of independent f64 MFMA chains vs fp64 VALU FMA chains.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_f64_probe mfma_f64_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// C = A x B (16x4 x 4x16) with lane maps A[l&15][l>>4], B[l>>4][l&15]; D[(l>>4)+4i][l&15].
// Then E = A2 x D  (D as B operand: k-step s uses register s), and F = D^T x B2 (D as A operand: register s).
__global__ void layout(const double* A, const double* B, const double* A2, const double* B2, double* C, double* E,
                       double* F) {
  const int l = threadIdx.x;
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[((l >> 4) + 4 * i) * 16 + (l & 15)] = acc[i];
  d4 e = {0, 0, 0, 0}, f = {0, 0, 0, 0};
  for (int s = 0; s < 4; ++s) {
    // A2 (16x16): A operand of k-step s = A2[l&15][4s + (l>>4)]; D row 4s+(l>>4) col l&15 = register s
    e = __builtin_amdgcn_mfma_f64_16x16x4f64(A2[(l & 15) * 16 + 4 * s + (l >> 4)], acc[s], e, 0, 0, 0);
    // D^T as A: A[m = l&15][k = 4s+(l>>4)] = D[4s+(l>>4)][l&15] = register s; B2[k][n] = B2[4s+(l>>4)][l&15]
    f = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[s], B2[(4 * s + (l >> 4)) * 16 + (l & 15)], f, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) {
    E[((l >> 4) + 4 * i) * 16 + (l & 15)] = e[i];
    F[((l >> 4) + 4 * i) * 16 + (l & 15)] = f[i];
  }
}

template <int CH>
__global__ __launch_bounds__(256) void mfma_tp(int iters, double* out) {
  const int l = threadIdx.x & 63;
  d4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = d4{0, 0, 0, 0};
  double a = 1.0 + l * 1e-3, b = 0.5 - l * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void valu_tp(int iters, double* out) {
  const int l = threadIdx.x & 63;
  double acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c;
  double a = 1.0 + l * 1e-9, b = 1e-9 * l;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], a, b);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

static double host_err(const double* got, const double* want, int n) {
  double e = 0;
  for (int i = 0; i < n; ++i) e = fmax(e, fabs(got[i] - want[i]));
  return e;
}

int main() {
  // ---- layout ----
  double hA[64], hB[64], hA2[256], hB2[256], hC[256], hE[256], hF[256], wC[256], wE[256], wF[256];
  for (int m = 0; m < 16; ++m) for (int k = 0; k < 4; ++k) hA[m * 4 + k] = (m * 7 + k * 3) % 11 - 5;
  for (int k = 0; k < 4; ++k) for (int n = 0; n < 16; ++n) hB[k * 16 + n] = (k * 5 + n * 2) % 9 - 4;
  for (int i = 0; i < 256; ++i) { hA2[i] = (i * 13) % 7 - 3; hB2[i] = (i * 17) % 5 - 2; }
  for (int m = 0; m < 16; ++m) for (int n = 0; n < 16; ++n) {
    double s = 0; for (int k = 0; k < 4; ++k) s += hA[m * 4 + k] * hB[k * 16 + n];
    wC[m * 16 + n] = s;
  }
  for (int m = 0; m < 16; ++m) for (int n = 0; n < 16; ++n) {
    double e = 0, f = 0;
    for (int k = 0; k < 16; ++k) { e += hA2[m * 16 + k] * wC[k * 16 + n]; f += wC[k * 16 + m] * hB2[k * 16 + n]; }
    wE[m * 16 + n] = e; wF[m * 16 + n] = f;
  }
  double *dA, *dB, *dA2, *dB2, *dC, *dE, *dF;
  CK(hipMalloc(&dA, 512)); CK(hipMalloc(&dB, 512)); CK(hipMalloc(&dA2, 2048)); CK(hipMalloc(&dB2, 2048));
  CK(hipMalloc(&dC, 2048)); CK(hipMalloc(&dE, 2048)); CK(hipMalloc(&dF, 2048));
  CK(hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA2, hA2, 2048, hipMemcpyHostToDevice)); CK(hipMemcpy(dB2, hB2, 2048, hipMemcpyHostToDevice));
  layout<<<1, 64>>>(dA, dB, dA2, dB2, dC, dE, dF);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hC, dC, 2048, hipMemcpyDeviceToHost)); CK(hipMemcpy(hE, dE, 2048, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hF, dF, 2048, hipMemcpyDeviceToHost));
  printf("layout C=AB max err %g | E=A2*C (C as B, reg s) %g | F=C^T*B2 (C as A, reg s) %g\n",
         host_err(hC, wC, 256), host_err(hE, wE, 256), host_err(hF, wF, 256));
  // ---- throughput ----
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8, iters = 20000;
  double* dout; CK(hipMalloc(&dout, (size_t)blocks * 256 * 8));
  hipEvent_t t0, t1; CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
  float ms;
  mfma_tp<8><<<blocks, 256>>>(100, dout); CK(hipDeviceSynchronize());
  CK(hipEventRecord(t0)); mfma_tp<8><<<blocks, 256>>>(iters, dout); CK(hipEventRecord(t1));
  CK(hipEventSynchronize(t1)); CK(hipEventElapsedTime(&ms, t0, t1));
  double waves = blocks * 4.0, mf = waves * iters * 8;
  printf("f64 MFMA 16x16x4: %.1f TFLOP/s  (%.1f ns per MFMA per SIMD, %d CUs)\n", mf * 2048 / (ms * 1e-3) / 1e12,
         ms * 1e6 / (mf / (cus * 4)), cus);
  valu_tp<8><<<blocks, 256>>>(100, dout); CK(hipDeviceSynchronize());
  CK(hipEventRecord(t0)); valu_tp<8><<<blocks, 256>>>(iters * 4, dout); CK(hipEventRecord(t1));
  CK(hipEventSynchronize(t1)); CK(hipEventElapsedTime(&ms, t0, t1));
  double fm = waves * iters * 4 * 8;
  printf("f64 VALU FMA: %.1f TFLOP/s  (%.2f ns per wave FMA per SIMD)\n", fm * 64 * 2 / (ms * 1e-3) / 1e12,
         ms * 1e6 / (fm / (cus * 4)));
  return 0;
}
