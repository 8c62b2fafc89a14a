// LDS atomic throughput probe (gfx950): cycles per wave-instruction for ds_add_f32 / ds_add_u32 / ds_write_b32
// at conflict-free lane-private addresses and at random bins, 8 waves per CU, 1 workgroup per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_atomic_bench lds_atomic_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE>
__global__ __launch_bounds__(512) void probe(int iters, float* out, uint32_t seed) {
  extern __shared__ float lh[];
  for (int i = threadIdx.x; i < 129 * 3 * 64; i += 512) lh[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 97u);
  float v = 1.0f;
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    const int b = (x >> 16) % 129;
    float* h = lh + b * 192 + lane;                  // lane-private layout [bin][stat][lane]
    if (MODE == 0) {
      atomicAdd(h, v); atomicAdd(h + 64, v); atomicAdd(h + 128, v);
    } else if (MODE == 1) {
      atomicAdd(reinterpret_cast<unsigned*>(h), 1u); atomicAdd(reinterpret_cast<unsigned*>(h) + 64, 1u);
      atomicAdd(reinterpret_cast<unsigned*>(h) + 128, 1u);
    } else if (MODE == 2) {
      h[0] = v; h[64] = v; h[128] = v;                // plain stores, same addresses
    } else if (MODE == 3) {
      float* hr = lh + (((x >> 8) & 127) * 3) + (lane & 0) ;   // random bins, shared histogram (row-per-lane style)
      atomicAdd(hr, v); atomicAdd(hr + 1, v); atomicAdd(hr + 2, v);
    } else if (MODE == 4) {
      // 64-bit integer adds, lanes split in two row halves of 32 features: [bin][stat][32] u64
      unsigned long long* hq = reinterpret_cast<unsigned long long*>(lh) + ((x >> 16) % 129) * 96 + (lane & 31);
      atomicAdd(hq, 3ull); atomicAdd(hq + 32, 5ull); atomicAdd(hq + 64, 7ull);
    } else if (MODE == 5) {
      double* hd = reinterpret_cast<double*>(lh) + ((x >> 16) % 129) * 96 + (lane & 31);
      atomicAdd(hd, 1.0); atomicAdd(hd + 32, 1.0); atomicAdd(hd + 64, 1.0);
    } else if (MODE == 6) {
      unsigned* hr = reinterpret_cast<unsigned*>(lh) + (((x >> 8) & 127) * 3);   // u32, shared random bins
      atomicAdd(hr, 1u); atomicAdd(hr + 1, 1u); atomicAdd(hr + 2, 1u);
    } else {
      // 32-bit integer adds, lanes split in two row halves: [bin][stat][64] with lane&31 + 32*half... same layout as 1
      unsigned* hu = reinterpret_cast<unsigned*>(lh) + ((x >> 16) % 129) * 192 + lane;
      atomicAdd(hu, 3u); atomicAdd(hu + 64, 5u); atomicAdd(hu + 128, 7u);
      atomicAdd(hu + 64 * 129 * 3 - 192 * 129 + 0, 0u);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lh[lane + 5];
}

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  float* out;
  hipMalloc(&out, sizeof(float) * cus * 8);
  const int iters = 20000;
  const size_t lds = 129 * 3 * 64 * 4;   // u64 modes use 32 lanes x 8 B: same bytes
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"ds_add_f32 lane-private", "ds_add_u32 lane-private", "ds_write_b32 lane-private",
                         "ds_add_f32 shared random bins", "ds_add_u64 32-lane-private", "ds_add_f64 32-lane-private",
                         "ds_add_u32 shared random bins"};
  for (int m = 0; m < 7; ++m) {
    void (*k)(int, float*, uint32_t) = m == 0 ? probe<0> : m == 1 ? probe<1> : m == 2 ? probe<2> : m == 3 ? probe<3>
                                     : m == 4 ? probe<4> : m == 5 ? probe<5> : probe<6>;
    hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(cus), dim3(512), lds, 0, 100, out, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(cus), dim3(512), lds, 0, iters, out, 7u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double instr_per_cu = 8.0 * iters * 3;     // 8 waves x iters x 3 wave-instructions
    printf("%-32s %8.3f ms  %.1f ns per wave-instruction per CU  (%.2f cycles @2.4GHz)\n", names[m], ms,
           ms * 1e6 / instr_per_cu, ms * 1e6 / instr_per_cu * 2.4);
  }
  hipFree(out);
  return 0;
}
