// Tree histogram kernels: hist[slot][feature][bin][stat] += stats[row][stat].
//
// Reference hot loops: ConstructLocalBin.java:135-166,209-240 (GBDT: per (node, feature, bin) sums of
// (g^2, g, h, 1) over fp64 arrays, one feature at a time on one CPU task) and TreeObj.stat
// (paralleltree/TreeObj.java:321-390; class-count / moment histograms for RF).
//
// CDNA4 design:
//  * bins are a row-major uint8 matrix [n, F] (one byte per (row, feature), <= 255 bins + a missing bin),
//    so consecutive lanes read consecutive feature bytes of a row: fully coalesced 256-byte wave loads.
//  * each workgroup owns a contiguous row range and a feature group; it privatises the
//    [slots x features x bins x stats] histogram in LDS as fp64 (ds_add_f64: ~9 cycles per wave-instruction on
//    gfx950 against ~193 for the native ds_add_f32 — see the K7 note at tree_hist_fm) and flushes non-zero
//    entries once with global fp32 atomics.  Per-(slot, feature) rows are padded by one element so lanes
//    working on neighbouring features land in different LDS banks.
//  * when even one feature of all slots does not fit the LDS budget the slots are split into groups
//    (grid.z); past 8 groups (very deep / wide levels, few rows per node) the kernel accumulates straight
//    into global memory instead, where contention is negligible.
//  * the host side builds only the smaller child of every split (histogram subtraction), so slot counts
//    stay at half the level width.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
constexpr int kLdsBudget = 64 * 1024;  // bytes per workgroup -> 2 workgroups per CU (160 KB LDS)

__global__ __launch_bounds__(kThreads) void tree_hist_lds(
    const uint8_t* __restrict__ bins, int64_t n, int F, const int32_t* __restrict__ slot,
    const float* __restrict__ stats, int S, int B, int slots_per_group, int FG, int64_t rows_per_block,
    float* __restrict__ hist) {
  extern __shared__ double sh[];   // fp64: ds_add_f64 ~9 cyc vs ds_add_f32 ~193 (K7 note below)
  const int fstride = B * S + 1;
  const int f0 = blockIdx.y * FG;
  const int fg = min(FG, F - f0);
  const int slot0 = blockIdx.z * slots_per_group;
  const int lds_n = slots_per_group * FG * fstride;
  for (int i = threadIdx.x; i < lds_n; i += kThreads) sh[i] = 0.0;
  __syncthreads();

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  if (r0 < r1) {
    const int npairs = (int)(r1 - r0) * fg;  // host guarantees < 2^31
    for (int p = threadIdx.x; p < npairs; p += kThreads) {
      const int rl = p / fg;
      const int f = p - rl * fg;
      const int64_t r = r0 + rl;
      const int s = slot[r] - slot0;
      if ((unsigned)s >= (unsigned)slots_per_group) continue;
      const int b = bins[r * F + f0 + f];
      double* h = sh + (s * FG + f) * fstride + b * S;
      const float* st = stats + r * S;
      for (int k = 0; k < S; ++k) {
        const float v = st[k];
        if (v != 0.f) atomicAdd(h + k, (double)v);
      }
    }
  }
  __syncthreads();

  // flush: LDS index i -> (slot s, local feature f, bin*S + k)
  const int bs = B * S;
  for (int i = threadIdx.x; i < lds_n; i += kThreads) {
    const float v = (float)sh[i];
    if (v == 0.f) continue;
    const int sf = i / fstride;
    const int rem = i - sf * fstride;
    if (rem >= bs) continue;  // padding column
    const int s = sf / FG;
    const int f = sf - s * FG;
    if (f >= fg || slot0 + s < 0) continue;
    const int64_t g = ((int64_t)(slot0 + s) * F + (f0 + f)) * bs + rem;
    unsafeAtomicAdd(hist + g, v);
  }
}

// Row-per-lane variant: a lane owns one row, keeps its S statistics in registers and walks the row's
// feature bytes; lanes of a wave hit the same feature at random bins (random LDS banks) and every row's
// stats/slot are loaded once instead of once per feature.
template <int S>
__global__ __launch_bounds__(kThreads) void tree_hist_rows(
    const uint8_t* __restrict__ bins, int64_t n, int F, const int32_t* __restrict__ slot,
    const float* __restrict__ stats, int B, int slots_per_group, int FG, int64_t rows_per_block,
    float* __restrict__ hist) {
  extern __shared__ double sh[];   // fp64: ds_add_f64 ~9 cyc vs ds_add_f32 ~193 (K7 note below)
  const int fstride = B * S + 1;
  const int f0 = blockIdx.y * FG;
  const int fg = min(FG, F - f0);
  const int slot0 = blockIdx.z * slots_per_group;
  const int lds_n = slots_per_group * FG * fstride;
  for (int i = threadIdx.x; i < lds_n; i += kThreads) sh[i] = 0.0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kThreads) {
    const int s = slot[r] - slot0;
    if ((unsigned)s >= (unsigned)slots_per_group) continue;
    double v[S];
#pragma unroll
    for (int k = 0; k < S; ++k) v[k] = (double)stats[r * S + k];
    const uint8_t* br = bins + r * F + f0;
    double* base = sh + s * FG * fstride;
    int f = 0;
    // 16 feature bytes per load when the row slice is 16-B aligned (F % 16 == 0, f0 % 16 == 0): one dwordx4
    // instead of 16 byte loads per lane
    if (((F | f0) & 15) == 0) {
      for (; f + 16 <= fg; f += 16) {
        const uint4 q = *reinterpret_cast<const uint4*>(br + f);
        const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          double* h = base + (f + j) * fstride + (int)((w4[j >> 2] >> (8 * (j & 3))) & 0xffu) * S;
#pragma unroll
          for (int k = 0; k < S; ++k) atomicAdd(h + k, v[k]);
        }
      }
    }
    for (; f < fg; ++f) {
      double* h = base + f * fstride + (int)br[f] * S;
#pragma unroll
      for (int k = 0; k < S; ++k) atomicAdd(h + k, v[k]);
    }
  }
  __syncthreads();
  const int bs = B * S;
  for (int i = threadIdx.x; i < lds_n; i += kThreads) {
    const float val = (float)sh[i];
    if (val == 0.f) continue;
    const int sf = i / fstride;
    const int rem = i - sf * fstride;
    if (rem >= bs) continue;
    const int s = sf / FG;
    const int f = sf - s * FG;
    if (f >= fg) continue;
    unsafeAtomicAdd(hist + ((int64_t)(slot0 + s) * F + (f0 + f)) * bs + rem, val);
  }
}

__global__ __launch_bounds__(kThreads) void tree_hist_global(
    const uint8_t* __restrict__ bins, int64_t n, int F, const int32_t* __restrict__ slot,
    const float* __restrict__ stats, int S, int B, int nslots, float* __restrict__ hist) {
  const int64_t total = n * (int64_t)F;
  const int bs = B * S;
  for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * kThreads) {
    const int64_t r = p / F;
    const int f = (int)(p - r * F);
    const int s = slot[r];
    if ((unsigned)s >= (unsigned)nslots) continue;
    const int b = bins[p];
    float* h = hist + ((int64_t)s * F + f) * bs + b * S;
    const float* st = stats + r * S;
    for (int k = 0; k < S; ++k) {
      const float v = st[k];
      if (v != 0.f) unsafeAtomicAdd(h + k, v);
    }
  }
}

// route rows one level down: child = base[node] + route[node][bin(row, feat[node])]
__global__ __launch_bounds__(kThreads) void tree_route(
    const uint8_t* __restrict__ bins, int64_t n, int F, int32_t* __restrict__ node,
    const int32_t* __restrict__ feat, const int32_t* __restrict__ base, const int16_t* __restrict__ route,
    int nnodes) {
  for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < n; r += (int64_t)gridDim.x * kThreads) {
    const int v = node[r];
    if ((unsigned)v >= (unsigned)nnodes) continue;
    const int f = feat[v];
    if (f < 0) {
      node[r] = base[v];  // leaf: host passes its final (negative) code
      continue;
    }
    const int b = bins[r * F + f];
    node[r] = base[v] + route[v * 256 + b];
  }
}

// Per-node statistic sums in fp64 (node counters: weight sum, count, g^2 ...): LDS-privatised ds_add_f64
// per workgroup, one global f64 atomic per (node, stat) per workgroup.  Rows with node outside [0, nnodes)
// or sample == 0 are skipped.
__global__ __launch_bounds__(kThreads) void tree_node_sums(const int32_t* __restrict__ node,
                                                           const uint8_t* __restrict__ sample,
                                                           const float* __restrict__ stats, int64_t n, int S,
                                                           int nnodes, int64_t rows_per_block,
                                                           double* __restrict__ out) {
  extern __shared__ double shd[];
  const int m = nnodes * S;
  for (int i = threadIdx.x; i < m; i += kThreads) shd[i] = 0.0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kThreads) {
    const int v = node[r];
    if ((unsigned)v >= (unsigned)nnodes || !sample[r]) continue;
    for (int k = 0; k < S; ++k) atomicAdd(shd + v * S + k, (double)stats[r * S + k]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += kThreads) {
    const double x = shd[i];
    if (x != 0.0) unsafeAtomicAdd(out + i, x);
  }
}

__global__ __launch_bounds__(kThreads) void tree_node_sums_global(const int32_t* __restrict__ node,
                                                                  const uint8_t* __restrict__ sample,
                                                                  const float* __restrict__ stats, int64_t n,
                                                                  int S, int nnodes, double* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < n; r += (int64_t)gridDim.x * kThreads) {
    const int v = node[r];
    if ((unsigned)v >= (unsigned)nnodes || !sample[r]) continue;
    for (int k = 0; k < S; ++k) unsafeAtomicAdd(out + (int64_t)v * S + k, (double)stats[r * S + k]);
  }
}

// ---------------------------------------------------------------------------------------------------------
// Fixed-point bank-private histogram (the production GPU path for S <= 4).
//
// Measured on MI355X (tools/micro/lds_atomic_bench.hip, 8 waves per CU): ds_add_f32 costs ~193 cycles per
// wave-instruction even with 64 distinct conflict-free addresses, ds_add_u32 ~6.  So the statistics are
// accumulated as 64-bit fixed point (integer LDS atomics): the host quantises every statistic column to int32
// with a power-of-two scale putting max|column| just below 2^30 (per-value resolution 2^-30 of the column's
// range, finer than an fp32 ulp of the typical sum), and the int64 bins cannot overflow below 2^33 rows.
// Integer sums are exact and order-independent: the histogram is bitwise deterministic and equal across
// partitionings of the rows.
//
// A workgroup owns one row chunk of ONE slot (rows pre-grouped by slot: ridx = row ids sorted stably by slot,
// q = their quantised statistics in that order, 4 x int32 per row) and one group of 32 features.  A wave
// takes rows in pairs: lanes 0-31 = features of row i, lanes 32-63 = the same features of row i+1; the LDS
// histogram is [bin][stat][32 features] int64, so each half-wave's 32 lanes hit 32 distinct, conflict-free
// 8-byte slots whatever the bins.  Row ids and statistics are wave-uniform scalar loads.
//
// XCD grouping: dispatch puts block ids b, b+8, b+16, b+24 on the same XCD at about the same time; they take
// the four 32-feature quarters of the same rows' 128-B cache lines.  Each block stores its partial histogram
// into an int64 slab (no global atomics, no zeroing); tree_hist_fm_reduce sums a slot's chunks and scales.
constexpr int kFmThreads = 1024;   // 16 waves: the single LDS-resident workgroup per CU hides HBM latency
constexpr int kFmPairs = 8;          // row pairs per batch and wave
// PACK (S == 3 with a unit count column, the GBDT / binary-RF case): the count rides in the low kPackBits of the
// first statistic's int64 — ((int64) q0 << kPackBits) + 1 per row, |q0| < 2^30 — so a (row, feature) pair costs
// 2 LDS atomics instead of 3 (the kernel is LDS-atomic-issue bound).  Exact while a chunk has < 2^kPackBits rows
// (the host caps chunks at kPackMaxRows): the q0 part then stays below 2^46 * 2^17 = 2^63 and the count never
// carries into it; tree_hist_fm_reduce unpacks every chunk's partial before summing chunks.
constexpr int kPackBits = 17;
constexpr int kPackMaxRows = 1 << 16;

template <int S, bool IDX, bool PACK = false>
__global__ __launch_bounds__(kFmThreads) void tree_hist_fm(const uint8_t* __restrict__ bins, int F,
                                                           const int32_t* __restrict__ ridx,
                                                           const int32_t* __restrict__ q,
                                                           const int32_t* __restrict__ chunk_rows, int nchunks,
                                                           const int32_t* __restrict__ fgl, int nfg, int B,
                                                           long long* __restrict__ slab) {
  extern __shared__ long long lq[];
  const int bid = blockIdx.x;
  const int nquad = (nfg + 3) >> 2;
  const int quad_id = (bid >> 5) * 8 + (bid & 7);
  const int c = quad_id / nquad;
  const int pos = (quad_id - c * nquad) * 4 + ((bid >> 3) & 3);   // entry of the feature-group list
  if (c >= nchunks || pos >= nfg) return;                // whole block, before any barrier
  const int fg = fgl != nullptr ? fgl[pos] : pos;
  constexpr int SL = PACK ? 2 : S;                       // int64 statistics per bin in LDS
  const int n_e = B * SL * 32;
  for (int i = threadIdx.x; i < n_e; i += kFmThreads) lq[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t f = (int64_t)fg * 32 + (lane & 31);      // fg may be a padding group far past F
  const bool valid = fg >= 0 && f < F;
  const uint8_t* bcol = bins + (valid ? f : 0);
  const int rb = chunk_rows[2 * c], re = chunk_rows[2 * c + 1];   // (start, end) pair: chunks may skip rows
  constexpr int nw = kFmThreads / 64;
  const int len = re - rb;
  const int per = ((len + nw - 1) / nw + 1) & ~1;        // even rows per wave
  const int i0 = rb + min(len, wave * per), i1 = rb + min(len, (wave + 1) * per);
  unsigned long long* lb = reinterpret_cast<unsigned long long*>(lq) + (lane & 31);
  const int bmax = B - 1;
  int i = i0;
  for (; i + 2 * kFmPairs <= i1; i += 2 * kFmPairs) {
    // row ids and both rows' statistics of every pair: wave-uniform scalar loads, issued together ahead of
    // the batch's LDS atomics (both count in lgkmcnt).  Per-lane vector loads of the statistics cost the
    // texture path 16 + 8 cycles per pair (64 lanes x 24 B, duplicates included) -- more than the atomics.
    int qs[kFmPairs][8];
    int bb[kFmPairs];
#pragma unroll
    for (int u = 0; u < kFmPairs; ++u) {
      const int64_t r0 = IDX ? (int64_t)ridx[i + 2 * u] : (int64_t)(i + 2 * u);
      const int64_t r1 = IDX ? (int64_t)ridx[i + 2 * u + 1] : (int64_t)(i + 2 * u + 1);
      bb[u] = bcol[(half ? r1 : r0) * F];
    }
#pragma unroll
    for (int u = 0; u < kFmPairs; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) qs[u][j] = q[(int64_t)(i + 2 * u) * 4 + j];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kFmPairs; ++u) {
      unsigned long long* hp = lb + min(bb[u], bmax) * (SL * 32);
      if (valid) {
        if constexpr (PACK) {
          // both rows' packed words are formed from the scalar statistics first (wave-uniform 64-bit values), and
          // the lane's half selects between them — selecting the int32 first made the compiler index qs and
          // spill it to scratch (10x slower)
          const long long p0 = ((long long)qs[u][0] << kPackBits) + 1, p1 = ((long long)qs[u][4] << kPackBits) + 1;
          const int h0 = qs[u][1], h1 = qs[u][5];
          const long long pv = half ? p1 : p0;
          const int hv = half ? h1 : h0;
          atomicAdd(hp, (unsigned long long)pv);
          atomicAdd(hp + 32, (unsigned long long)(long long)hv);
        } else {
#pragma unroll
          for (int k = 0; k < S; ++k) {
            const int lo = qs[u][k], hi = qs[u][4 + k];     // select by value: an index would go to scratch
            const int v = half ? hi : lo;
            atomicAdd(hp + k * 32, (unsigned long long)(long long)v);
          }
        }
      }
    }
  }
  for (; i < i1; i += 2) {
    const bool has1 = i + 1 < i1;
    const int64_t r0 = IDX ? (int64_t)ridx[i] : (int64_t)i;
    const int64_t r1 = has1 ? (IDX ? (int64_t)ridx[i + 1] : (int64_t)(i + 1)) : r0;
    const int b = bcol[(half ? r1 : r0) * F];
    unsigned long long* hp = lb + min(b, bmax) * (SL * 32);
    if (valid && (half == 0 || has1)) {
      if constexpr (PACK) {
        atomicAdd(hp, (unsigned long long)(((long long)q[(int64_t)(i + half) * 4] << kPackBits) + 1));
        atomicAdd(hp + 32, (unsigned long long)(long long)q[(int64_t)(i + half) * 4 + 1]);
      } else {
#pragma unroll
        for (int k = 0; k < S; ++k)
          atomicAdd(hp + k * 32, (unsigned long long)(long long)q[(int64_t)(i + half) * 4 + k]);
      }
    }
  }
  __syncthreads();
  long long* dst = slab + ((int64_t)c * nfg + pos) * n_e;
  for (int j = threadIdx.x; j < n_e; j += kFmThreads) dst[j] = lq[j];
}

// H[slot][fg*32 + l][b][k] = inv_scale[k] * sum over the slot's chunks of slab[chunk][pos][b][k][l] (exact int64
// sums), fg = fgl[pos]; feature-major mode writes Hfm[pos*32 + l][slot][b][k] instead (every row, zeros for
// features >= F: the layout a per-rank reduce-scatter sends).  A block owns (slot, list entry, 8 bins) and
// transposes through LDS (row stride 33: conflict-free).
constexpr int kRedBins = 8;
__global__ __launch_bounds__(256) void tree_hist_fm_reduce(const long long* __restrict__ slab,
                                                           const int32_t* __restrict__ slot_chunk,
                                                           const int32_t* __restrict__ fgl, int nfg, int nslots,
                                                           int F, int B, int S, const double* __restrict__ inv_scale,
                                                           int feat_major, float* __restrict__ H, int pack) {
  __shared__ float tile[kRedBins * 4 * 33];
  const int s = blockIdx.x / nfg, pos = blockIdx.x - (blockIdx.x / nfg) * nfg;
  const int fg = fgl != nullptr ? fgl[pos] : pos;
  const int b0 = blockIdx.y * kRedBins;
  const int nb = min(kRedBins, B - b0);
  const int cs = slot_chunk[s], ce = slot_chunk[s + 1];
  if (pack) {
    // slab holds [B][2][32]: (q0 << kPackBits) + count, q1.  Every chunk's packed word is split before the chunks
    // are summed (the count field is exact per chunk only); output statistics 0, 1 scaled, 2 = the count.
    const int n_e = B * 2 * 32;
    const int m = nb * 2 * 32;
    for (int t = threadIdx.x; t < m; t += 256) {
      long long acc = 0, cnt = 0;
      const bool first = ((t >> 5) & 1) == 0;
      for (int j = cs; j < ce; ++j) {
        const long long v = slab[((int64_t)j * nfg + pos) * n_e + (int64_t)b0 * 2 * 32 + t];
        if (first) {
          acc += v >> kPackBits;
          cnt += v & ((1ll << kPackBits) - 1);
        } else {
          acc += v;
        }
      }
      const int bl = t >> 6, l = t & 31;
      if (first) {
        tile[(bl * 3 + 0) * 33 + l] = (float)((double)acc * inv_scale[0]);
        tile[(bl * 3 + 2) * 33 + l] = (float)cnt;
      } else {
        tile[(bl * 3 + 1) * 33 + l] = (float)((double)acc * inv_scale[1]);
      }
    }
  } else {
    const int n_e = B * S * 32;
    const int m = nb * S * 32;
    for (int t = threadIdx.x; t < m; t += 256) {
      long long acc = 0;
      for (int j = cs; j < ce; ++j) acc += slab[((int64_t)j * nfg + pos) * n_e + (int64_t)b0 * S * 32 + t];
      const int k = (t >> 5) % S;
      tile[(t >> 5) * 33 + (t & 31)] = (float)((double)acc * inv_scale[k]);
    }
  }
  __syncthreads();
  const int w = nb * S;
  for (int t = threadIdx.x; t < 32 * w; t += 256) {
    const int l = t / w, j = t - (t / w) * w;
    if (feat_major) {
      H[(((int64_t)(pos * 32 + l) * nslots + s) * B + b0) * S + j] = tile[j * 33 + l];
    } else {
      const int64_t f = (int64_t)fg * 32 + l;
      if (fg >= 0 && f < F) H[(((int64_t)s * F + f) * B + b0) * S + j] = tile[j * 33 + l];
    }
  }
}

// Row gather of the tree's node-grouped order (RowOrder.regroup / the per-call sort path): dst_q[i] = src_q[p[i]]
// (16-byte rows of four int32 statistics, one int4 load + store per thread) and dst_o[i] = src_o[p[i]] when src_o
// is given.  torch's generic index kernel moved these 16-byte rows at ~0.2 TB/s.
__global__ __launch_bounds__(256) void tree_gather_rows_kernel(const int4* __restrict__ src_q,
                                                              const int32_t* __restrict__ src_o,
                                                              const int64_t* __restrict__ p, int64_t n,
                                                              int4* __restrict__ dst_q, int32_t* __restrict__ dst_o) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = p[i];
    dst_q[i] = src_q[j];
    if (src_o != nullptr) dst_o[i] = src_o[j];
  }
}

template <int S, bool PACK = false>
int launch_fm(bool idx, int64_t grid, size_t lds, hipStream_t stream, const uint8_t* bins, int F, const int32_t* ridx,
              const int32_t* sst, const int32_t* chunk_rows, int nchunks, const int32_t* fgl, int nfg, int B,
              long long* slab) {
  const void* k = idx ? reinterpret_cast<const void*>(tree_hist_fm<S, true, PACK>)
                      : reinterpret_cast<const void*>(tree_hist_fm<S, false, PACK>);
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return 3;
  if (idx)
    hipLaunchKernelGGL((tree_hist_fm<S, true, PACK>), dim3((unsigned)grid), dim3(kFmThreads), lds, stream, bins, F,
                       ridx, sst, chunk_rows, nchunks, fgl, nfg, B, slab);
  else
    hipLaunchKernelGGL((tree_hist_fm<S, false, PACK>), dim3((unsigned)grid), dim3(kFmThreads), lds, stream, bins, F,
                       ridx, sst, chunk_rows, nchunks, fgl, nfg, B, slab);
  return 0;
}

}  // namespace

extern "C" {

// out: [nnodes, S] fp64, zeroed by the caller.
int alink_tree_node_sums(const int32_t* node, const uint8_t* sample, const float* stats, int64_t n, int S,
                         int nnodes, double* out, int num_cus, hipStream_t stream) {
  if (n <= 0 || nnodes <= 0) return 0;
  const size_t lds = (size_t)nnodes * S * sizeof(double);
  if (lds <= 64 * 1024) {
    int64_t target = (int64_t)num_cus * 4;
    int64_t rpb = (n + target - 1) / target;
    if (rpb < 4096) rpb = 4096;
    const int64_t gx = (n + rpb - 1) / rpb;
    hipLaunchKernelGGL(tree_node_sums, dim3((unsigned)gx), dim3(kThreads), lds, stream, node, sample, stats, n, S,
                       nnodes, rpb, out);
  } else {
    int64_t blocks = (n + kThreads - 1) / kThreads;
    int grid = (int)(blocks < (int64_t)num_cus * 8 ? blocks : (int64_t)num_cus * 8);
    hipLaunchKernelGGL(tree_node_sums_global, dim3(grid), dim3(kThreads), 0, stream, node, sample, stats, n, S,
                       nnodes, out);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}


// hist must be zeroed by the caller: [nslots, F, B, S] fp32.
// variant bit 0: use the (row, feature)-pair kernel instead of the row-per-lane kernel.
int alink_tree_hist_f32(const uint8_t* bins, int64_t n, int F, const int32_t* slot, const float* stats,
                        int S, int B, int nslots, float* hist, int num_cus, int variant, hipStream_t stream) {
  if (n <= 0 || nslots <= 0) return 0;
  if (F <= 0 || S <= 0 || B <= 0 || B > 256) return 1;
  const int unit = (B * S + 1) * (int)sizeof(double);  // one (slot, feature) row of the fp64 LDS table
  const int max_units = kLdsBudget / unit;
  int FG, spg, groups;
  if (max_units >= nslots) {
    spg = nslots;
    groups = 1;
    FG = max_units / nslots;
    if (FG > F) FG = F;
    if (FG >= 16 && FG < F) FG &= ~15;   // 16-feature aligned groups -> vector bin loads in tree_hist_rows
  } else {
    FG = 1;
    spg = max_units > 0 ? max_units : 1;
    groups = (nslots + spg - 1) / spg;
  }
  if (max_units == 0 || groups > 8) {
    int64_t total = n * (int64_t)F;
    int64_t blocks = (total + kThreads - 1) / kThreads;
    int grid = (int)(blocks < (int64_t)num_cus * 16 ? blocks : (int64_t)num_cus * 16);
    hipLaunchKernelGGL(tree_hist_global, dim3(grid), dim3(kThreads), 0, stream, bins, n, F, slot, stats, S, B,
                       nslots, hist);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  const int gy = (F + FG - 1) / FG;
  // ~4 workgroups per CU overall; each needs enough rows to amortise its LDS clear + flush
  int64_t target = (int64_t)num_cus * 4 / ((int64_t)gy * groups);
  if (target < 1) target = 1;
  int64_t rows_per_block = (n + target - 1) / target;
  const int64_t min_rows = 2048;
  if (rows_per_block < min_rows) rows_per_block = min_rows;
  const int64_t max_rows = ((int64_t)1 << 30) / (FG > 0 ? FG : 1);
  if (rows_per_block > max_rows) rows_per_block = max_rows;
  const int64_t gx = (n + rows_per_block - 1) / rows_per_block;
  const size_t lds = (size_t)spg * FG * unit;
  const dim3 grid((unsigned)gx, gy, groups);
  if (S >= 2 && S <= 4 && !(variant & 1)) {
    if (S == 2)
      hipLaunchKernelGGL(tree_hist_rows<2>, grid, dim3(kThreads), lds, stream, bins, n, F, slot, stats, B, spg, FG,
                         rows_per_block, hist);
    else if (S == 3)
      hipLaunchKernelGGL(tree_hist_rows<3>, grid, dim3(kThreads), lds, stream, bins, n, F, slot, stats, B, spg, FG,
                         rows_per_block, hist);
    else
      hipLaunchKernelGGL(tree_hist_rows<4>, grid, dim3(kThreads), lds, stream, bins, n, F, slot, stats, B, spg, FG,
                         rows_per_block, hist);
  } else {
    hipLaunchKernelGGL(tree_hist_lds, grid, dim3(kThreads), lds, stream, bins, n, F, slot, stats, S, B, spg, FG,
                       rows_per_block, hist);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// dst_q[i] = src_q[p[i]] (int32 [., 4] rows), dst_o[i] = src_o[p[i]] (src_o / dst_o nullable), i < n.
int alink_tree_gather_rows(const int32_t* src_q, const int32_t* src_o, const int64_t* p, int64_t n, int32_t* dst_q,
                           int32_t* dst_o, hipStream_t stream) {
  if (n <= 0) return 0;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(tree_gather_rows_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, stream,
                     reinterpret_cast<const int4*>(src_q), src_o, p, n, reinterpret_cast<int4*>(dst_q), dst_o);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Fixed-point histogram (tree_hist_fm): rows grouped by slot.  ridx: [total] row ids sorted by slot (nullptr =
// identity: rows 0..total-1 all in slot 0); q: [total, 4] int32 quantised statistics in that order;
// chunk_rows: [nchunks][2] (start, end) row offsets (each chunk inside one slot; rows between chunks are
// skipped: the tree's node-grouped row order holds the rows of derived / finished nodes too); slot_chunk:
// [nslots+1] chunk ranges per
// slot; fgl: [nfl] 32-feature groups to build (nullptr: all, nfl ignored); inv_scale: [S] fp64 (device);
// slab: [nchunks, nfl, B, S, 32] int64 scratch; H: [nslots, F, B, S] fp32, or with feat_major
// [nfl * 32, nslots, B, S] (fully written, no zeroing needed).
// pack = 1 (S == 3, statistic 2 a unit count; every chunk < kPackMaxRows rows): the packed 2-atomic build.
int alink_tree_hist_fm(const uint8_t* bins, int F, const int32_t* ridx, const int32_t* q, const int32_t* chunk_rows,
                       int nchunks, const int32_t* slot_chunk, int nslots, int S, int B, const int32_t* fgl, int nfl,
                       int feat_major, const double* inv_scale, long long* slab, float* H, hipStream_t stream,
                       int pack) {
  if (nslots <= 0) return 0;
  if (F <= 0 || S < 1 || S > 4 || B <= 0 || B > 256 || (pack && S != 3)) return 1;
  const size_t lds = (size_t)B * (pack ? 2 : S) * 32 * sizeof(long long);
  if (lds > 160 * 1024) return 1;
  const int nfg = fgl != nullptr ? nfl : (F + 31) / 32;
  if (nfg <= 0) return 0;
  if (nchunks > 0) {
    const int64_t quads = (int64_t)nchunks * ((nfg + 3) / 4);
    const int64_t grid = (quads + 7) / 8 * 32;
    if (grid > 0x7fffffff) return 1;
    const int rc = pack ? launch_fm<3, true>(ridx != nullptr, grid, lds, stream, bins, F, ridx, q, chunk_rows, nchunks, fgl, nfg, B, slab)
                 : S == 1 ? launch_fm<1>(ridx != nullptr, grid, lds, stream, bins, F, ridx, q, chunk_rows, nchunks, fgl, nfg, B, slab)
                 : S == 2 ? launch_fm<2>(ridx != nullptr, grid, lds, stream, bins, F, ridx, q, chunk_rows, nchunks, fgl, nfg, B, slab)
                 : S == 3 ? launch_fm<3>(ridx != nullptr, grid, lds, stream, bins, F, ridx, q, chunk_rows, nchunks, fgl, nfg, B, slab)
                          : launch_fm<4>(ridx != nullptr, grid, lds, stream, bins, F, ridx, q, chunk_rows, nchunks, fgl, nfg, B, slab);
    if (rc != 0) return rc;
  }
  hipLaunchKernelGGL(tree_hist_fm_reduce, dim3((unsigned)(nslots * nfg), (unsigned)((B + kRedBins - 1) / kRedBins)),
                     dim3(256), 0, stream, slab, slot_chunk, fgl, nfg, nslots, F, B, S, inv_scale, feat_major, H, pack);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// node: int32 [n] current node index within the level (>= nnodes or < 0: already finished, untouched).
// feat: [nnodes] split feature (-1 = leaf); base: [nnodes] first child index in the next level (for a leaf:
// the negative code the row keeps from now on);
// route: [nnodes, 256] child offset per bin.
int alink_tree_route(const uint8_t* bins, int64_t n, int F, int32_t* node, const int32_t* feat,
                     const int32_t* base, const int16_t* route, int nnodes, int num_cus, hipStream_t stream) {
  if (n <= 0) return 0;
  int64_t blocks = (n + kThreads - 1) / kThreads;
  int grid = (int)(blocks < (int64_t)num_cus * 8 ? blocks : (int64_t)num_cus * 8);
  hipLaunchKernelGGL(tree_route, dim3(grid), dim3(kThreads), 0, stream, bins, n, F, node, feat, base, route,
                     nnodes);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
