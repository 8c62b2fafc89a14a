// Feature hot path on CDNA4 (gfx950 / MI355X): Guava-exact murmur3 feature hashing (K26) and the per-row CSR
// assembler behind FeatureHasher / OneHot / VectorAssembler (K24/K25).
//
//   * murmur3: one lane per string, Guava Murmur3_32HashFunction(0).hashUnencodedChars over UTF-16 code units
//     (chars taken in pairs, low unit first; odd tail unit mixed alone; fmix with 2 * length) of the virtual
//     string prefix ++ value, so "col=" + value needs no host concatenation.  Output: floorMod(abs(h), nf) with
//     Java int semantics (abs(INT_MIN) stays negative) — reference FeatureHasherMapper.java:104-106.
//   * CSR assembler: one 64-lane wave per row, lane j holds the row's entry from input column j (m <= 64):
//     bitonic sort by (index, column) in registers (__shfl_xor), duplicate indices merged by a segmented suffix
//     scan (TreeMap.put(index, old + value) of the reference), heads compacted with a ballot prefix count.
//     Two passes (count -> host cumsum -> write) give row-sorted, unique-index CSR directly on the device.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ __forceinline__ uint32_t mix_k1(uint32_t k1) {
    k1 *= 0xcc9e2d51u;
    k1 = rotl32(k1, 15);
    return k1 * 0x1b873593u;
}

__device__ __forceinline__ uint32_t mix_h1(uint32_t h1, uint32_t k1) {
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    return h1 * 5u + 0xe6546b64u;
}

__device__ __forceinline__ uint32_t fmix(uint32_t h1, uint32_t len_bytes) {
    h1 ^= len_bytes;
    h1 ^= h1 >> 16;
    h1 *= 0x85ebca6bu;
    h1 ^= h1 >> 13;
    h1 *= 0xc2b2ae35u;
    h1 ^= h1 >> 16;
    return h1;
}

__global__ __launch_bounds__(256) void murmur3_index_kernel(const uint16_t* __restrict__ units,
                                                           const int64_t* __restrict__ off, int64_t n,
                                                           const uint16_t* __restrict__ prefix, int plen,
                                                           uint32_t seed, int64_t nf, int32_t* __restrict__ hash_out,
                                                           int32_t* __restrict__ index_out) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = off[s];
        const int64_t len = (int64_t)plen + (off[s + 1] - b);
        auto ch = [&](int64_t j) -> uint32_t { return j < plen ? prefix[j] : units[b + j - plen]; };
        uint32_t h1 = seed;
        for (int64_t i = 1; i < len; i += 2) h1 = mix_h1(h1, mix_k1(ch(i - 1) | (ch(i) << 16)));
        if (len & 1) h1 ^= mix_k1(ch(len - 1));
        const int32_t h = (int32_t)fmix(h1, (uint32_t)(2 * len));
        if (hash_out != nullptr) hash_out[s] = h;
        if (index_out != nullptr) {
            const int64_t a = h == INT32_MIN ? (int64_t)INT32_MIN : (h < 0 ? -(int64_t)h : (int64_t)h);
            int64_t r = a % nf;                          // Math.floorMod(int, int)
            if (r < 0) r += nf;
            index_out[s] = (int32_t)r;
        }
    }
}

// UTF-8 input: lane decodes its string's code points and feeds the UTF-16 code units (surrogate pairs above
// U+FFFF) to the same pairwise mixing, so a packed UTF-8 StringBlock hashes Guava-exactly with no host pass.
struct U16Mixer {
    uint32_t h1, pending;
    int64_t n;  // code units so far
    __device__ __forceinline__ void push(uint32_t u) {
        if (n & 1) h1 = mix_h1(h1, mix_k1(pending | (u << 16)));
        else pending = u;
        ++n;
    }
    __device__ __forceinline__ uint32_t finish() {
        if (n & 1) h1 ^= mix_k1(pending);
        return fmix(h1, (uint32_t)(2 * n));
    }
};

__device__ __forceinline__ void push_utf8(U16Mixer& m, const uint8_t* __restrict__ p, int64_t len) {
    for (int64_t i = 0; i < len;) {
        const uint32_t b0 = p[i];
        uint32_t cp;
        if (b0 < 0x80u) {
            cp = b0;
            i += 1;
        } else if (b0 < 0xE0u && i + 1 < len) {
            cp = ((b0 & 0x1Fu) << 6) | (p[i + 1] & 0x3Fu);
            i += 2;
        } else if (b0 < 0xF0u && i + 2 < len) {
            cp = ((b0 & 0x0Fu) << 12) | ((p[i + 1] & 0x3Fu) << 6) | (p[i + 2] & 0x3Fu);
            i += 3;
        } else if (i + 3 < len) {
            cp = ((b0 & 0x07u) << 18) | ((p[i + 1] & 0x3Fu) << 12) | ((p[i + 2] & 0x3Fu) << 6) | (p[i + 3] & 0x3Fu);
            i += 4;
        } else {
            cp = 0xFFFDu;  // truncated sequence (not produced by Python's encoder)
            i += 1;
        }
        if (cp >= 0x10000u) {
            const uint32_t c = cp - 0x10000u;
            m.push(0xD800u + (c >> 10));
            m.push(0xDC00u + (c & 0x3FFu));
        } else {
            m.push(cp);
        }
    }
}

__global__ __launch_bounds__(256) void murmur3_utf8_index_kernel(const uint8_t* __restrict__ bytes,
                                                                const int64_t* __restrict__ off, int64_t n,
                                                                const uint16_t* __restrict__ prefix, int plen,
                                                                uint32_t seed, int64_t nf,
                                                                int32_t* __restrict__ hash_out,
                                                                int32_t* __restrict__ index_out) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
        U16Mixer m{seed, 0u, 0};
        for (int j = 0; j < plen; ++j) m.push(prefix[j]);
        const int64_t b = off[s];
        push_utf8(m, bytes + b, off[s + 1] - b);
        const int32_t h = (int32_t)m.finish();
        if (hash_out != nullptr) hash_out[s] = h;
        if (index_out != nullptr) {
            const int64_t a = h == INT32_MIN ? (int64_t)INT32_MIN : (h < 0 ? -(int64_t)h : (int64_t)h);
            int64_t r = a % nf;
            if (r < 0) r += nf;
            index_out[s] = (int32_t)r;
        }
    }
}

// Several packed string columns at once (FeatureHasher over m categorical fields): column j's strings hashed with
// its own "name=" prefix into row j of idx [m][n] (int32 feature index) and valid [m][n] (uint8, 0 for NULL).
// The column table travels BY VALUE in the kernel arguments: one launch per micro-batch instead of ~6 per column,
// and no host->device copy of descriptors.
constexpr int kMhMaxCols = 32;
constexpr int kMhMaxPrefix = 1024;
struct MultiHashArgs {
    const uint8_t* data[kMhMaxCols];
    const int64_t* off[kMhMaxCols];
    const uint8_t* nulls[kMhMaxCols];      // bool bytes, nullptr = no NULLs
    int32_t pstart[kMhMaxCols + 1];        // prefix of column j = prefix[pstart[j] .. pstart[j+1])
    uint16_t prefix[kMhMaxPrefix];
};

__global__ __launch_bounds__(256) void murmur3_multi_index_kernel(const MultiHashArgs a, int m, int64_t n,
                                                                 uint32_t seed, int64_t nf,
                                                                 int32_t* __restrict__ idx,
                                                                 uint8_t* __restrict__ valid) {
    const int64_t total = (int64_t)m * n;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(t / n);
        const int64_t r = t - (int64_t)j * n;
        const bool ok = a.nulls[j] == nullptr || a.nulls[j][r] == 0;
        U16Mixer mx{seed, 0u, 0};
        for (int q = a.pstart[j]; q < a.pstart[j + 1]; ++q) mx.push(a.prefix[q]);
        const int64_t b = a.off[j][r];
        push_utf8(mx, a.data[j] + b, a.off[j][r + 1] - b);
        const int32_t h = (int32_t)mx.finish();
        const int64_t ab = h == INT32_MIN ? (int64_t)INT32_MIN : (h < 0 ? -(int64_t)h : (int64_t)h);
        int64_t q = ab % nf;
        if (q < 0) q += nf;
        idx[t] = ok ? (int32_t)q : 0;
        valid[t] = ok ? 1 : 0;
    }
}

// MurmurHash3_x86_32 over raw bytes (Guava murmur3_32().hashBytes): shuffle keys of packed string columns.
__global__ __launch_bounds__(256) void murmur3_bytes_kernel(const uint8_t* __restrict__ bytes,
                                                           const int64_t* __restrict__ off, int64_t n, uint32_t seed,
                                                           int32_t* __restrict__ out) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = off[s], len = off[s + 1] - b;
        const uint8_t* p = bytes + b;
        uint32_t h1 = seed;
        const int64_t nb = len >> 2;
        for (int64_t i = 0; i < nb; ++i) {
            const uint32_t k = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
                               ((uint32_t)p[4 * i + 3] << 24);
            h1 = mix_h1(h1, mix_k1(k));
        }
        uint32_t k1 = 0;
        const uint8_t* t = p + 4 * nb;
        switch (len & 3) {
            case 3: k1 ^= (uint32_t)t[2] << 16; [[fallthrough]];
            case 2: k1 ^= (uint32_t)t[1] << 8; [[fallthrough]];
            case 1: k1 ^= t[0]; h1 ^= mix_k1(k1);
        }
        out[s] = (int32_t)fmix(h1, (uint32_t)len);
    }
}

constexpr int32_t KEY_NONE = 0x7fffffff;

// sort (key, tag) ascending across the wave with the value riding along; tag = input column (stable order)
__device__ __forceinline__ void wave_bitonic_sort(int32_t& key, int32_t& tag, double& v, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int32_t ok = __shfl_xor(key, j);
            const int32_t ot = __shfl_xor(tag, j);
            const double ov = __shfl_xor(v, j);
            const bool up = (lane & k) == 0;                 // ascending block
            const bool lower = (lane & j) == 0;              // this lane keeps the smaller of the pair
            const bool other_less = ok < key || (ok == key && ot < tag);
            const bool take = lower == up ? other_less : !other_less;
            if (take) {
                key = ok;
                tag = ot;
                v = ov;
            }
        }
    }
}

// one row per wave: returns (in registers) the sorted, merged entry of this lane and whether it is a head
__device__ __forceinline__ bool row_entries(int64_t r, int64_t n, int m, const int32_t* __restrict__ idx,
                                            const double* __restrict__ val, const uint8_t* __restrict__ valid,
                                            int lane, int32_t& key, double& sum) {
    int32_t k = KEY_NONE, tag = lane;
    double v = 0.0;
    if (lane < m) {
        const int64_t p = (int64_t)lane * n + r;
        if (valid == nullptr || valid[p]) {
            k = idx[p];
            v = val != nullptr ? val[p] : 1.0;
        }
    }
    wave_bitonic_sort(k, tag, v, lane);
    // segmented suffix sum over runs of equal keys (sorted -> runs are contiguous)
    double s = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double t = __shfl_down(s, o);
        const int32_t k2 = __shfl_down(k, o);
        if (lane + o < 64 && k2 == k) s += t;
    }
    const int32_t kp = __shfl_up(k, 1);
    key = k;
    sum = s;
    return k != KEY_NONE && (lane == 0 || kp != k);
}

__global__ __launch_bounds__(256) void csr_count_kernel(int64_t n, int m, const int32_t* __restrict__ idx,
                                                       const uint8_t* __restrict__ valid, int64_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r = w0; r < n; r += nw) {
        int32_t key;
        double s;
        const bool head = row_entries(r, n, m, idx, nullptr, valid, lane, key, s);
        const uint64_t heads = __ballot(head);
        if (lane == 0) cnt[r] = __popcll(heads);
    }
}

__global__ __launch_bounds__(256) void csr_write_kernel(int64_t n, int m, const int32_t* __restrict__ idx,
                                                       const double* __restrict__ val,
                                                       const uint8_t* __restrict__ valid,
                                                       const int64_t* __restrict__ crow, int32_t* __restrict__ col,
                                                       double* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r = w0; r < n; r += nw) {
        int32_t key;
        double s;
        const bool head = row_entries(r, n, m, idx, val, valid, lane, key, s);
        const uint64_t heads = __ballot(head);
        const int pos = __popcll(heads & ((1ull << lane) - 1ull));
        if (head) {
            col[crow[r] + pos] = key;
            out[crow[r] + pos] = s;
        }
    }
}

// CSR matrix-vector product out[r] = sum_k val[k] * v[col[k]] over row r's entries (FeatureMatrix.mv: linear /
// FTRL margins).  G lanes per row (G a power of two <= 64 picked from the mean row length), each lane a strided
// run of the row's entries, then a fixed-order xor-shuffle tree within the group: deterministic, no atomics
// (torch's index_add_ of the per-entry products serialises on the rows' addresses).
template <int G, typename I>
__global__ __launch_bounds__(256) void csr_mv_kernel(const int64_t* __restrict__ crow, const I* __restrict__ col,
                                                    const double* __restrict__ val, int64_t nrows,
                                                    const double* __restrict__ v, double* __restrict__ out) {
    const int sub = threadIdx.x & (G - 1);
    const int64_t g0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    const int64_t ng = (int64_t)gridDim.x * blockDim.x / G;
    // r is uniform across a group's G lanes, so a group enters and leaves the loop together (shuffle-safe)
    for (int64_t r = g0; r < nrows; r += ng) {
        const int64_t s = crow[r], e = crow[r + 1];
        double acc = 0.0;
        for (int64_t k = s + sub; k < e; k += G) acc = fma(val[k], v[(int64_t)col[k]], acc);
#pragma unroll
        for (int o = G >> 1; o > 0; o >>= 1) acc += __shfl_xor(acc, o, G);
        if (sub == 0) out[r] = acc;
    }
}

// VectorAssembler (K24, reference VectorAssemblerMapper.java:50-106): every output row is the concatenation of
// its parts' entries, each shifted by the running position (dense parts contribute every value, zeros included;
// sparse parts their stored entries), so the CSR row is sorted by construction.  One thread per (part, row):
// threads of a wave take consecutive rows of one part (coalesced reads of the part), find their run's offset
// in the output row from the earlier parts' run lengths, and copy the run.  A NULL row (handleInvalid SKIP,
// decided on the host) contributes nothing.  Part descriptor (8 x int64 per part):
//   kind (0 dense fp64, 1 dense fp32, 2 dense bf16, 3 CSR fp64), width (dense: columns; CSR: vector size),
//   val ptr, crow ptr (CSR), col ptr (CSR, int32), nulls ptr (uint8, nullable), position of the part's first
//   column in the output vector, 0.
__device__ __forceinline__ int64_t part_len(const int64_t* __restrict__ d, int64_t r) {
    const uint8_t* nulls = reinterpret_cast<const uint8_t*>(d[5]);
    if (nulls != nullptr && nulls[r]) return 0;
    if (d[0] == 3) {
        const int64_t* crow = reinterpret_cast<const int64_t*>(d[3]);
        return crow[r + 1] - crow[r];
    }
    return d[1];
}

__global__ __launch_bounds__(256) void vector_assemble_kernel(int64_t n, int P, const int64_t* __restrict__ desc,
                                                             const int64_t* __restrict__ out_crow,
                                                             int32_t* __restrict__ out_col,
                                                             double* __restrict__ out_val) {
    const int64_t total = n * P;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(t / n);
        const int64_t r = t - (int64_t)p * n;
        const int64_t* d = desc + 8 * p;
        const int64_t L = part_len(d, r);
        if (L == 0) continue;
        int64_t o = out_crow[r];
        for (int q = 0; q < p; ++q) o += part_len(desc + 8 * q, r);
        const int64_t pos = d[6];
        const int kind = (int)d[0];
        if (kind == 3) {
            const int64_t s = reinterpret_cast<const int64_t*>(d[3])[r];
            const int32_t* col = reinterpret_cast<const int32_t*>(d[4]) + s;
            const double* val = reinterpret_cast<const double*>(d[2]) + s;
            for (int64_t j = 0; j < L; ++j) {
                out_col[o + j] = (int32_t)(pos + col[j]);
                out_val[o + j] = val[j];
            }
        } else {
            const int64_t base = r * L;
            for (int64_t j = 0; j < L; ++j) {
                double v;
                if (kind == 0) v = reinterpret_cast<const double*>(d[2])[base + j];
                else if (kind == 1) v = (double)reinterpret_cast<const float*>(d[2])[base + j];
                else v = (double)__uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(d[2])[base + j] << 16);
                out_col[o + j] = (int32_t)(pos + j);
                out_val[o + j] = v;
            }
        }
    }
}

// VectorAssembler v2 (P <= 16 parts): one 256-thread workgroup per 256 rows.  Thread t first forms row r0+t's
// run offsets per part (LDS), then the workgroup walks its contiguous output range element by element: each
// thread finds its element's row by binary search over the LDS row starts and its part by a scan of the row's
// run offsets, reads the source entry and writes col / val -- consecutive threads write consecutive entries
// (coalesced stores; v1 wrote one row-run per thread, 64 scattered runs per store instruction).
constexpr int kVaRows = 256;
constexpr int kVaMaxP = 16;

__global__ __launch_bounds__(256) void vector_assemble_v2_kernel(int64_t n, int P, const int64_t* __restrict__ desc,
                                                                const int64_t* __restrict__ out_crow,
                                                                int32_t* __restrict__ out_col,
                                                                double* __restrict__ out_val) {
  __shared__ int32_t roff[kVaMaxP + 1][kVaRows];        // run start of part p inside row t (p = P: row length)
  __shared__ int32_t rstart[kVaRows + 1];              // row start inside the workgroup's output range
  __shared__ int64_t d_s[kVaMaxP * 8];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kVaRows;
  const int nr = (int)min((int64_t)kVaRows, n - r0);
  for (int i = t; i < P * 8; i += 256) d_s[i] = desc[i];
  __syncthreads();
  const int64_t base = out_crow[r0];
  if (t < nr) {
    int32_t o = 0;
    for (int p = 0; p < P; ++p) {
      roff[p][t] = o;
      o += (int32_t)part_len(d_s + 8 * p, r0 + t);
    }
    roff[P][t] = o;
    rstart[t] = (int32_t)(out_crow[r0 + t] - base);
  }
  if (t == 0) rstart[nr] = (int32_t)(out_crow[r0 + nr] - base);
  __syncthreads();
  const int32_t total = rstart[nr];
  for (int32_t e = t; e < total; e += 256) {
    int lo = 0, hi = nr;                                 // last row with rstart <= e
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (rstart[mid] <= e) lo = mid;
      else hi = mid;
    }
    const int row = lo;
    const int32_t j = e - rstart[row];
    int p = 0;
    while (p + 1 < P && roff[p + 1][row] <= j) ++p;
    const int64_t* d = d_s + 8 * p;
    const int64_t k = j - roff[p][row];
    const int64_t r = r0 + row;
    const int kind = (int)d[0];
    int32_t c;
    double v;
    if (kind == 3) {
      const int64_t s = reinterpret_cast<const int64_t*>(d[3])[r] + k;
      c = (int32_t)(d[6] + reinterpret_cast<const int32_t*>(d[4])[s]);
      v = reinterpret_cast<const double*>(d[2])[s];
    } else {
      const int64_t src = r * d[1] + k;
      c = (int32_t)(d[6] + k);
      if (kind == 0) v = reinterpret_cast<const double*>(d[2])[src];
      else if (kind == 1) v = (double)reinterpret_cast<const float*>(d[2])[src];
      else v = (double)__uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(d[2])[src] << 16);
    }
    out_col[base + e] = c;
    out_val[base + e] = v;
  }
}

}  // namespace

extern "C" {

// floorMod(abs(murmur3_32(seed).hashUnencodedChars(prefix + s_i)), nf) for n strings given as UTF-16 code units
// (units, off[n+1]); hash_out / index_out nullable.
int alink_murmur3_index(const uint16_t* units, const int64_t* off, int64_t n, const uint16_t* prefix, int plen,
                        uint32_t seed, int64_t nf, int32_t* hash_out, int32_t* index_out, void* stream) {
    if (n <= 0) return 0;
    if (nf <= 0 || plen < 0) return 1;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(murmur3_index_kernel, dim3(blocks < 8192 ? blocks : 8192), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), units, off, n, prefix, plen, seed, nf, hash_out,
                       index_out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// As alink_murmur3_index for strings given as packed UTF-8 (bytes, off[n+1]): UTF-16 units decoded in-lane.
int alink_murmur3_utf8_index(const uint8_t* bytes, const int64_t* off, int64_t n, const uint16_t* prefix, int plen,
                             uint32_t seed, int64_t nf, int32_t* hash_out, int32_t* index_out, void* stream) {
    if (n <= 0) return 0;
    if (nf <= 0 || plen < 0) return 1;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(murmur3_utf8_index_kernel, dim3(blocks < 8192 ? blocks : 8192), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), bytes, off, n, prefix, plen, seed, nf, hash_out,
                       index_out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// m <= 32 packed string columns hashed in one launch (args: a host MultiHashArgs, copied into the kernel
// arguments); idx / valid [m][n] device outputs.
int alink_murmur3_multi_index(const void* args, int m, int64_t n, uint32_t seed, int64_t nf, int32_t* idx,
                              uint8_t* valid, void* stream) {
    if (n <= 0 || m <= 0) return 0;
    if (m > kMhMaxCols || nf <= 0) return 1;
    const MultiHashArgs a = *reinterpret_cast<const MultiHashArgs*>(args);
    if (a.pstart[m] > kMhMaxPrefix) return 1;
    const int64_t blocks = ((int64_t)m * n + 255) / 256;
    hipLaunchKernelGGL(murmur3_multi_index_kernel, dim3(blocks < 16384 ? blocks : 16384), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), a, m, n, seed, nf, idx, valid);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// MurmurHash3_x86_32(seed) of every packed byte string (bytes, off[n+1]) -> out[n].
int alink_murmur3_bytes(const uint8_t* bytes, const int64_t* off, int64_t n, uint32_t seed, int32_t* out,
                        void* stream) {
    if (n <= 0) return 0;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(murmur3_bytes_kernel, dim3(blocks < 8192 ? blocks : 8192), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), bytes, off, n, seed, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// VectorAssembler rows: desc [P][8] int64 part descriptors (device), out_crow [n+1] (host-computed prefix of
// the per-row entry counts), out_col / out_val [out_crow[n]].  variant 2: element-parallel workgroups (P <= 16,
// rows shorter than 2^22 entries), else one thread per (part, row).
int alink_vector_assemble(int64_t n, int P, const int64_t* desc, const int64_t* out_crow, int32_t* out_col,
                          double* out_val, int variant, void* stream) {
    if (n <= 0 || P <= 0) return 0;
    if (P <= kVaMaxP && variant == 2) {
        const int64_t nb = (n + kVaRows - 1) / kVaRows;
        hipLaunchKernelGGL(vector_assemble_v2_kernel, dim3((unsigned)nb), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), n, P, desc, out_crow, out_col, out_val);
        return hipGetLastError() == hipSuccess ? 0 : 2;
    }
    const int64_t blocks = (n * P + 255) / 256;
    hipLaunchKernelGGL(vector_assemble_kernel, dim3(blocks < 65536 ? blocks : 65536), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), n, P, desc, out_crow, out_col, out_val);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// CSR rows from m <= 64 column-major entry arrays idx/val/valid [m][n] (val nullable -> 1.0, valid nullable ->
// all valid): pass 1 (out == nullptr) writes cnt[n]; pass 2 writes col/out at crow (cumsum of cnt).
// out[nrows] = CSR(crow, col, val) @ v; col int32 (idx64 = 0) or int64 (idx64 = 1); mean_nnz picks lanes per row
int alink_csr_mv_f64(const int64_t* crow, const void* col, int idx64, const double* val, int64_t nrows,
                     const double* v, double* out, double mean_nnz, void* stream) {
    if (nrows <= 0) return 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int G = mean_nnz > 48 ? 64 : mean_nnz > 24 ? 32 : mean_nnz > 12 ? 16 : mean_nnz > 6 ? 8 : 4;
    const int64_t groups = nrows;
    int64_t blocks = (groups * G + 255) / 256;
    if (blocks > 8192) blocks = 8192;
#define ALINK_CSR_MV(GG)                                                                                          \
    if (G == GG) {                                                                                                \
        if (idx64)                                                                                                \
            hipLaunchKernelGGL((csr_mv_kernel<GG, int64_t>), dim3(blocks), dim3(256), 0, st, crow,                \
                               reinterpret_cast<const int64_t*>(col), val, nrows, v, out);                        \
        else                                                                                                      \
            hipLaunchKernelGGL((csr_mv_kernel<GG, int32_t>), dim3(blocks), dim3(256), 0, st, crow,                \
                               reinterpret_cast<const int32_t*>(col), val, nrows, v, out);                        \
    }
    ALINK_CSR_MV(4) ALINK_CSR_MV(8) ALINK_CSR_MV(16) ALINK_CSR_MV(32) ALINK_CSR_MV(64)
#undef ALINK_CSR_MV
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

int alink_csr_assemble(int64_t n, int m, const int32_t* idx, const double* val, const uint8_t* valid, int64_t* cnt,
                       const int64_t* crow, int32_t* col, double* out, void* stream) {
    if (n <= 0) return 0;
    if (m < 1 || m > 64) return 1;
    const int64_t blocks = (n + 3) / 4;
    const dim3 grid(blocks < 16384 ? blocks : 16384);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (out == nullptr)
        hipLaunchKernelGGL(csr_count_kernel, grid, dim3(256), 0, st, n, m, idx, valid, cnt);
    else
        hipLaunchKernelGGL(csr_write_kernel, grid, dim3(256), 0, st, n, m, idx, val, valid, crow, col, out);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
