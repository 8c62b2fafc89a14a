// Hogwild FTRL-proximal on CDNA4 (gfx950 / MI355X) for high-throughput online logistic regression.
//
// Same per-coordinate rule as the reference's CalcTask (FtrlTrainStreamOp.java:396-485) and the sequential host
// loop (_native/csrc/ftrl.cpp):
//   g = (p - y) x_i;  sigma = (sqrt(n_i + g^2) - sqrt(n_i)) / alpha;  z_i += g - sigma w_i;  n_i += g^2
//   w_i = |z_i| <= l1 ? 0 : (sign(z_i) l1 - z_i) / (beta + sqrt(n_i)/alpha + l2)
// but the samples of a micro-batch are processed CONCURRENTLY, one 64-wide wave per sample (grid-strided):
// the wave's lanes stride over the sample's non-zeros, the margin w.x is a wave reduction, then every lane
// updates its coordinates with fp64 atomics.  n_i and z_i are updated by device-scope atomicAdd (executed at
// the memory side, so exact across the 8 XCDs) and w_i is recomputed from the values the atomics returned:
// concurrent updates to one coordinate never lose a gradient.  Only the w_i a sample READS may be stale (the
// per-XCD L2s are not coherent) -- the Hogwild relaxation.  The reference has the same staleness: its margin is
// computed in flatMap1 (:396-420) before the feedback of earlier samples reaches flatMap2 (:423-485).  Exact
// when the samples in flight touch disjoint coordinates.  Opt-in (updateMode = HOGWILD); the sequential mode
// stays the default because it is run-to-run deterministic.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr int THREADS = 256;
constexpr int WAVES = THREADS / 64;

__device__ __forceinline__ double ld_relaxed(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(THREADS) void ftrl_hogwild_kernel(const int64_t* __restrict__ indptr,
                                                              const int32_t* __restrict__ idx,
                                                              const double* __restrict__ val,
                                                              const double* __restrict__ label, int64_t nrows,
                                                              double* w, double* n, double* z, double alpha,
                                                              double beta, double l1, double l2) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * WAVES;
    for (int64_t r = wave; r < nrows; r += nwaves) {
        const int64_t s = indptr[r], e = indptr[r + 1];
        double wx = 0.0;
        for (int64_t k = s + lane; k < e; k += 64) wx = fma(val[k], ld_relaxed(&w[idx[k]]), wx);
        for (int off = 32; off > 0; off >>= 1) wx += __shfl_xor(wx, off);
        const double p = 1.0 / (1.0 + exp(-wx));
        const double err = p - label[r];
        for (int64_t k = s + lane; k < e; k += 64) {
            const int32_t i = idx[k];
            const double g = err * val[k];
            const double g2 = g * g;
            const double wi = ld_relaxed(&w[i]);
            const double n_old = atomicAdd(&n[i], g2);
            const double n_new = n_old + g2;
            const double sigma = (sqrt(n_new) - sqrt(n_old)) / alpha;
            const double dz = g - sigma * wi;
            const double z_new = atomicAdd(&z[i], dz) + dz;
            const double wn = fabs(z_new) <= l1
                                  ? 0.0
                                  : ((z_new < 0 ? -1.0 : 1.0) * l1 - z_new) / (beta + sqrt(n_new) / alpha + l2);
            __hip_atomic_store(&w[i], wn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Feature-sharded micro-batch FTRL (updateMode SHARDED; reference FtrlTrainStreamOp.java:174-267
// SplitVector, :396-420 partial margins, :488-567 keyed reduce + feedback).  Rank r owns coordinates [lo, hi).
//   1. partial margin of every sample of the (all-gathered) micro-batch on the owned range (one wave per row);
//      the host all-reduces the margins over the ranks;
//   2. every owned coordinate replays its entries in sample order (entries pre-sorted by coordinate, stable):
//      one lane per coordinate, the recurrence is sequential per coordinate and independent across them, so
//      the result does not depend on the number of ranks or on thread scheduling (deterministic).
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void ftrl_partial_margin_kernel(const int64_t* __restrict__ indptr,
                                                                     const int32_t* __restrict__ idx,
                                                                     const double* __restrict__ val, int64_t nrows,
                                                                     const double* __restrict__ w, int64_t lo,
                                                                     int64_t hi, double* __restrict__ margin) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * WAVES;
    for (int64_t r = wave; r < nrows; r += nwaves) {
        const int64_t s = indptr[r], e = indptr[r + 1];
        double wx = 0.0;
        for (int64_t k = s + lane; k < e; k += 64) {
            const int64_t i = idx[k];
            if (i >= lo && i < hi) wx = fma(val[k], w[i - lo], wx);
        }
        for (int off = 32; off > 0; off >>= 1) wx += __shfl_xor(wx, off);
        if (lane == 0) margin[r] = wx;
    }
}

// seg[nseg+1]: boundaries into the coordinate-sorted entry order; g[t] = err[row] * x (gathered for the
// sorted order in one parallel pass beforehand), coord[q] = the segment's coordinate.  The serial part is then
// a walk over a contiguous g run: the n / sqrt / denominator chain does not depend on z, so unrolled steps
// overlap it with the z recurrence.  State arrays are the owned shard (index - lo).
__global__ __launch_bounds__(256) void ftrl_coord_update_kernel(const int64_t* __restrict__ seg, int64_t nseg,
                                                               const int64_t* __restrict__ nseg_dev,
                                                               const int64_t* __restrict__ coord,
                                                               const double* __restrict__ g, double* w, double* n,
                                                               double* z, int64_t lo, int64_t hi, double alpha,
                                                               double beta, double l1, double l2, int64_t maxlen) {
    const double ia = 1.0 / alpha;
    const int64_t ns = nseg_dev != nullptr ? *nseg_dev : nseg;   // device-side count: no host sync to size it
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < ns; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = seg[q], e = seg[q + 1];
        if (e - s > maxlen) continue;                 // ftrl_coord_long_kernel's segment
        if (coord[q] >= hi) continue;                 // entries of coordinates this shard does not own
        const int64_t i = coord[q] - lo;
        double wi = w[i], ni = n[i], zi = z[i], sq = sqrt(ni);
        // The only serial dependence is z -> w -> z: sigma_t and the prox denominator depend on n alone (a prefix
        // sum of g^2), so their sqrt / reciprocal sit off the chain and the unrolled loop overlaps them with
        // earlier steps; the chain itself is two FMAs, a compare/select and a multiply per step (it was a full
        // fp64 IEEE division per step: a hot coordinate such as the intercept is a 65536-step chain per batch).
#pragma unroll 8
        for (int64_t t = s; t < e; ++t) {
            const double gt = g[t];
            const double nn = ni + gt * gt;
            const double sn = sqrt(nn);
            const double sigma = (sn - sq) * ia;
            const double rden = 1.0 / (beta + sn * ia + l2);
            zi += gt - sigma * wi;
            ni = nn;
            sq = sn;
            wi = fabs(zi) <= l1 ? 0.0 : (copysign(l1, zi) - zi) * rden;
        }
        w[i] = wi;
        n[i] = ni;
        z[i] = zi;
    }
}

// Long segments (hot coordinates: the intercept is in every sample) get a whole wave, 64 entries per chunk: the
// lanes load g coalesced, form n_t by a wave prefix sum of g^2 and compute sigma_t and the prox reciprocal r_t in
// parallel.  The z -> w chain is then speculated: while sign(z) and |z| > l1 do not change, prox is affine in z,
// so each step is an affine map z_t = a_t z_{t-1} + b_t (a_t = 1 + sigma_t r_{t-1}, b_t = g_t - sigma_t sgn l1
// r_{t-1}; a_t = 1, b_t = g_t in the |z| <= l1 regime) and the chunk is a wave prefix scan of map compositions.
// The regime is guessed from the chunk's first step (computed exactly from the carried w) and checked on every
// z_{t-1}; a chunk whose z crosses a regime boundary replays step by step with the per-step operands broadcast
// by v_readlane.  (A single lane walking a 65536-step intercept segment cost ~190 ns per step; the serial
// broadcast replay ~76 ns; the scan ~6 steps of 64-lane shuffles per 64 entries.)
__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double prox_r(double zv, double l1, double r) {
    return fabs(zv) <= l1 ? 0.0 : (copysign(l1, zv) - zv) * r;
}

__device__ __forceinline__ int regime(double zv, double l1) { return fabs(zv) <= l1 ? 0 : (zv > 0.0 ? 1 : -1); }

// entries [s, e) of one coordinate from the carried (wi, ni, zi), one 64-lane wave (lane = threadIdx.x & 63; every
// lane of the wave must call it); the final state is returned in (wi, ni, zi) on every lane
__device__ void long_chain(const double* __restrict__ g, int64_t s, int64_t e, int lane, double ia, double beta,
                           double l1, double l2, double& wi, double& ni, double& zi) {
    for (int64_t t0 = s; t0 < e; t0 += 64) {
        const int cnt = (int)(e - t0 < 64 ? e - t0 : 64);
        const double gl = lane < cnt ? g[t0 + lane] : 0.0;
        double ps = gl * gl;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double o = __shfl_up(ps, d);
            if (lane >= d) ps += o;
        }
        // every shuffle runs with all lanes active (a bpermute from a lane masked off by a branch reads 0)
        const double nl = ni + ps;
        const double snl = sqrt(nl);
        const double up = __shfl_up(snl, 1);
        const double sprev = lane == 0 ? sqrt(ni) : up;
        const double sig = (snl - sprev) * ia;
        const double rden = 1.0 / (beta + snl * ia + l2);
        const double rprev = __shfl_up(rden, 1);
        // step 0 is exact from the carried w; its result fixes the guessed regime of the chunk
        const double z0 = zi + gl - sig * wi;                       // meaningful on lane 0
        const int guess = regime(readlane_d(z0, 0), l1);
        double am, bm;
        if (lane == 0) {
            am = 1.0;
            bm = gl - sig * wi;
        } else if (lane < cnt && guess != 0) {
            am = 1.0 + sig * rprev;
            bm = gl - sig * (guess * l1) * rprev;
        } else {
            am = 1.0;
            bm = lane < cnt ? gl : 0.0;
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const double ao = __shfl_up(am, d), bo = __shfl_up(bm, d);
            if (lane >= d) {
                bm = fma(am, bo, bm);
                am *= ao;
            }
        }
        const double zl = fma(am, zi, bm);                           // z after this lane's step
        const double zprev = __shfl_up(zl, 1);
        const bool bad = lane >= 1 && lane < cnt && regime(zprev, l1) != guess;
        if (__ballot(bad) == 0) {
            zi = readlane_d(zl, cnt - 1);
            wi = prox_r(zi, l1, readlane_d(rden, cnt - 1));
        } else {
            for (int u = 0; u < cnt; ++u) {
                const double gu = readlane_d(gl, u), su = readlane_d(sig, u), ru = readlane_d(rden, u);
                zi += gu - su * wi;
                wi = prox_r(zi, l1, ru);
            }
        }
        ni = readlane_d(nl, cnt - 1);
    }
}

__global__ __launch_bounds__(64) void ftrl_coord_long_kernel(const int64_t* __restrict__ seg,
                                                            const int64_t* __restrict__ coord,
                                                            const int64_t* __restrict__ lsegs, int64_t nlong,
                                                            const int64_t* __restrict__ nlong_dev,
                                                            const double* __restrict__ g, double* w, double* n,
                                                            double* z, int64_t lo, double alpha, double beta,
                                                            double l1, double l2) {
    const int lane = threadIdx.x;
    const int64_t cnt = nlong_dev != nullptr ? *nlong_dev : nlong;
    for (int64_t li = blockIdx.x; li < cnt; li += gridDim.x) {
        const int64_t q = lsegs[li];
        const int64_t i = coord[q] - lo;
        double wi = w[i], ni = n[i], zi = z[i];
        long_chain(g, seg[q], seg[q + 1], lane, 1.0 / alpha, beta, l1, l2, wi, ni, zi);
        if (lane == 0) {
            w[i] = wi;
            n[i] = ni;
            z[i] = zi;
        }
    }
}

// Very long segments (the intercept: every sample of the micro-batch) as ONE speculative scan over the whole
// segment on a 512-thread block instead of 64-entry chunks walked in sequence (~1 us per chunk: 1.1 ms per
// 65536-sample batch).  Thread t owns a contiguous run of ceil(len / 512) entries:
//   pass 1  sum of g^2 over the run -> block exclusive scan -> n before the run (n_t is a prefix sum of g^2);
//   pass 2  per entry sigma_t, r_t (prox reciprocal) from n alone, the entry's affine map under the regime guessed
//           from the exact first step (as in ftrl_coord_long_kernel), composed over the run -> block exclusive
//           scan of map compositions -> z before the run;
//   pass 3  the run's z_t replayed from there, every z_{t-1} checked against the guessed regime.
// If every check passes, the final (w, n, z) come from the last entry; otherwise the state just before the FIRST
// failing entry is exact, and wave 0 finishes the segment from it with the chunked walk (long_chain).
constexpr int SCAN_NT = 512;

struct Aff {
    double a, b;                                  // z -> a z + b
};

__device__ __forceinline__ Aff aff_then(Aff first, Aff second) {   // second(first(z))
    return Aff{second.a * first.a, fma(second.a, first.b, second.b)};
}

// block exclusive prefix (sum) of one double per thread; sh: SCAN_NT / 64 doubles
__device__ double block_excl_sum(double v, double* sh) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(x, d);
        if (lane >= d) x += o;
    }
    const double ex = __shfl_up(x, 1);
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    double off = 0.0;
    for (int k = 0; k < wv; ++k) off += sh[k];
    __syncthreads();
    return off + (lane == 0 ? 0.0 : ex);
}

// block exclusive prefix of affine maps (composition in thread order); sa / sb: SCAN_NT / 64 doubles each
__device__ Aff block_excl_aff(Aff v, double* sa, double* sb) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    Aff x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const Aff o{__shfl_up(x.a, d), __shfl_up(x.b, d)};
        if (lane >= d) x = aff_then(o, x);
    }
    const Aff ex{__shfl_up(x.a, 1), __shfl_up(x.b, 1)};
    if (lane == 63) {
        sa[wv] = x.a;
        sb[wv] = x.b;
    }
    __syncthreads();
    Aff off{1.0, 0.0};
    for (int k = 0; k < wv; ++k) off = aff_then(off, Aff{sa[k], sb[k]});
    __syncthreads();
    return lane == 0 ? off : aff_then(off, ex);
}

struct ScanShared {
    double a[SCAN_NT / 64], b[SCAN_NT / 64];
    long long bad;
    double z, n;
};

__device__ void scan_segment(ScanShared& sm, int64_t q, const int64_t* __restrict__ seg,
                             const int64_t* __restrict__ coord, const double* __restrict__ g, double* w, double* n,
                             double* z, int64_t lo, double alpha, double beta, double l1, double l2) {
    double* sh_a = sm.a;
    double* sh_b = sm.b;
    long long& sh_bad = sm.bad;
    double& sh_z = sm.z;
    double& sh_n = sm.n;
    const int tid = threadIdx.x;
    const int64_t s = seg[q], e = seg[q + 1];
    const int64_t i = coord[q] - lo;
    const double ia = 1.0 / alpha;
    const double w0 = w[i], n0 = n[i], z0 = z[i];
    const int64_t per = (e - s + SCAN_NT - 1) / SCAN_NT;
    const int64_t rs = s + tid * per < e ? s + tid * per : e, re = rs + per < e ? rs + per : e;
    if (tid == 0) sh_bad = (long long)e;
    // the regime of z after the exact first step
    int guess;
    {
        const double g0 = g[s];
        const double sig0 = (sqrt(n0 + g0 * g0) - sqrt(n0)) * ia;
        guess = regime(z0 + g0 - sig0 * w0, l1);
    }
    // pass 1: n before the run
    double gs = 0.0;
    for (int64_t t = rs; t < re; ++t) gs = fma(g[t], g[t], gs);
    const double nrun = n0 + block_excl_sum(gs, sh_a);
    // pass 2: the run's composed map
    Aff m{1.0, 0.0};
    {
        double nn = nrun, sq = sqrt(nrun), rprev = 1.0 / (beta + sq * ia + l2);
        for (int64_t t = rs; t < re; ++t) {
            const double gt = g[t];
            nn += gt * gt;
            const double sn = sqrt(nn);
            const double sig = (sn - sq) * ia;
            Aff st;
            if (t == s) st = Aff{1.0, gt - sig * w0};
            else if (guess != 0) st = Aff{1.0 + sig * rprev, gt - sig * (guess * l1) * rprev};
            else st = Aff{1.0, gt};
            m = aff_then(m, st);
            sq = sn;
            rprev = 1.0 / (beta + sn * ia + l2);
        }
    }
    const Aff pre = block_excl_aff(m, sh_a, sh_b);
    // pass 3: replay and check
    {
        double zp = fma(pre.a, z0, pre.b), nn = nrun, sq = sqrt(nrun), rprev = 1.0 / (beta + sq * ia + l2);
        for (int64_t t = rs; t < re; ++t) {
            if (t > s && regime(zp, l1) != guess) {          // first failing entry of this run
                atomicMin(&sh_bad, (long long)t);
                break;
            }
            const double gt = g[t];
            nn += gt * gt;
            const double sn = sqrt(nn);
            const double sig = (sn - sq) * ia;
            Aff st;
            if (t == s) st = Aff{1.0, gt - sig * w0};
            else if (guess != 0) st = Aff{1.0 + sig * rprev, gt - sig * (guess * l1) * rprev};
            else st = Aff{1.0, gt};
            zp = fma(st.a, zp, st.b);
            sq = sn;
            rprev = 1.0 / (beta + sn * ia + l2);
        }
    }
    __syncthreads();
    const int64_t bad = (int64_t)sh_bad;
    if (bad == e) {
        if (re == e && re > rs) {                             // the thread holding the last entry
            double zp = fma(pre.a, z0, pre.b), nn = nrun, sq = sqrt(nrun), rprev = 1.0 / (beta + sq * ia + l2);
            for (int64_t t = rs; t < re; ++t) {              // replay once more (registers hold no history)
                const double gt = g[t];
                nn += gt * gt;
                const double sn = sqrt(nn);
                const double sig = (sn - sq) * ia;
                Aff st;
                if (t == s) st = Aff{1.0, gt - sig * w0};
                else if (guess != 0) st = Aff{1.0 + sig * rprev, gt - sig * (guess * l1) * rprev};
                else st = Aff{1.0, gt};
                zp = fma(st.a, zp, st.b);
                sq = sn;
                rprev = 1.0 / (beta + sn * ia + l2);
            }
            z[i] = zp;
            n[i] = nn;
            w[i] = prox_r(zp, l1, rprev);
        }
        return;
    }
    // state just before entry `bad` (> s): the thread whose run holds bad - 1 replays up to it
    if (rs < re && bad - 1 >= rs && bad - 1 < re) {
        double zp = fma(pre.a, z0, pre.b), nn = nrun, sq = sqrt(nrun), rprev = 1.0 / (beta + sq * ia + l2);
        for (int64_t t = rs; t < bad; ++t) {
            const double gt = g[t];
            nn += gt * gt;
            const double sn = sqrt(nn);
            const double sig = (sn - sq) * ia;
            Aff st;
            if (t == s) st = Aff{1.0, gt - sig * w0};
            else if (guess != 0) st = Aff{1.0 + sig * rprev, gt - sig * (guess * l1) * rprev};
            else st = Aff{1.0, gt};
            zp = fma(st.a, zp, st.b);
            sq = sn;
            rprev = 1.0 / (beta + sn * ia + l2);
        }
        sh_z = zp;
        sh_n = nn;
    }
    __syncthreads();
    if (tid < 64) {
        double zi = sh_z, ni = sh_n;
        double wi = prox_r(zi, l1, 1.0 / (beta + sqrt(ni) * ia + l2));
        long_chain(g, bad, e, tid, ia, beta, l1, l2, wi, ni, zi);
        if (tid == 0) {
            w[i] = wi;
            n[i] = ni;
            z[i] = zi;
        }
    }
}

__global__ __launch_bounds__(SCAN_NT) void ftrl_coord_scan_kernel(const int64_t* __restrict__ seg,
                                                                const int64_t* __restrict__ coord,
                                                                const int64_t* __restrict__ lsegs, int64_t nlong,
                                                                const int64_t* __restrict__ nlong_dev,
                                                                const double* __restrict__ g, double* w, double* n,
                                                                double* z, int64_t lo, double alpha, double beta,
                                                                double l1, double l2) {
    __shared__ ScanShared sm;
    const int64_t cnt = nlong_dev != nullptr ? *nlong_dev : nlong;
    for (int64_t li = blockIdx.x; li < cnt; li += gridDim.x) {
        scan_segment(sm, lsegs[li], seg, coord, g, w, n, z, lo, alpha, beta, l1, l2);
        __syncthreads();                              // the shared state is reused by the next segment
    }
}

// w_i = prox(z_i, n_i) for the listed coordinates (all when coords == nullptr): makes the Hogwild weights
// consistent with the exact n/z sums after a contended micro-batch (the racing w stores are last-writer-wins).
__global__ __launch_bounds__(256) void ftrl_prox_kernel(const int32_t* __restrict__ coords, int64_t m, double* w,
                                                       const double* __restrict__ n, const double* __restrict__ z,
                                                       double alpha, double beta, double l1, double l2) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = coords != nullptr ? (int64_t)coords[q] : q;
        const double zi = z[i];
        w[i] = fabs(zi) <= l1 ? 0.0 : ((zi < 0 ? -1.0 : 1.0) * l1 - zi) / (beta + sqrt(n[i]) / alpha + l2);
    }
}

__global__ void ftrl_check_kernel(const int32_t* __restrict__ idx, int64_t nnz, int64_t dim, int* __restrict__ bad) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x)
        if (idx[k] < 0 || idx[k] >= dim) atomicOr(bad, 1);
}

}  // namespace

extern "C" {

// Validates every feature index against dim (bad[0] != 0 afterwards when one is out of range).  The caller runs
// it and checks bad before alink_ftrl_hogwild_f64: the update kernel trusts its indices.
int alink_ftrl_check_indices(const int32_t* idx, int64_t nnz, int64_t dim, int* bad, int grid, void* stream) {
    if (nnz <= 0) return 0;
    hipLaunchKernelGGL(ftrl_check_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), idx, nnz, dim, bad);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

int alink_ftrl_hogwild_f64(const int64_t* indptr, const int32_t* idx, const double* val, const double* label,
                           int64_t nrows, double* w, double* n, double* z, double alpha, double beta, double l1,
                           double l2, int grid, void* stream) {
    if (nrows <= 0) return 0;
    if (grid <= 0 || alpha <= 0.0) return 1;
    hipLaunchKernelGGL(ftrl_hogwild_kernel, dim3(grid), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                       indptr, idx, val, label, nrows, w, n, z, alpha, beta, l1, l2);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

int alink_ftrl_partial_margin_f64(const int64_t* indptr, const int32_t* idx, const double* val, int64_t nrows,
                                  const double* w, int64_t lo, int64_t hi, double* margin, int grid, void* stream) {
    if (nrows <= 0) return 0;
    if (grid <= 0 || hi < lo) return 1;
    hipLaunchKernelGGL(ftrl_partial_margin_kernel, dim3(grid), dim3(THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                       indptr, idx, val, nrows, w, lo, hi, margin);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// nseg_dev (nullable): the segment count read on the device (nseg is then only the launch's upper bound);
// coordinates >= hi are skipped (entries the shard does not own, sorted to the end)
int alink_ftrl_coord_update_f64(const int64_t* seg, int64_t nseg, const int64_t* nseg_dev, const int64_t* coord,
                                const double* g, double* w, double* n, double* z, int64_t lo, int64_t hi,
                                double alpha, double beta, double l1, double l2, int64_t maxlen, int grid,
                                void* stream) {
    if (nseg <= 0) return 0;
    if (grid <= 0 || alpha <= 0.0) return 1;
    hipLaunchKernelGGL(ftrl_coord_update_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), seg,
                       nseg, nseg_dev, coord, g, w, n, z, lo, hi, alpha, beta, l1, l2, maxlen);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// segments of SCAN_MIN entries or more: one 512-thread speculative scan each (ftrl_coord_scan_kernel)
// nlong_dev (nullable): the list length read on the device; the launch then has `grid` blocks striding over it
int alink_ftrl_coord_scan_f64(const int64_t* seg, const int64_t* coord, const int64_t* lsegs, int64_t nlong,
                              const int64_t* nlong_dev, const double* g, double* w, double* n, double* z, int64_t lo,
                              double alpha, double beta, double l1, double l2, int grid, void* stream) {
    if (nlong <= 0) return 0;
    const unsigned gb = nlong_dev != nullptr ? (unsigned)(grid > 0 ? grid : 1) : (unsigned)nlong;
    hipLaunchKernelGGL(ftrl_coord_scan_kernel, dim3(gb), dim3(SCAN_NT), 0, reinterpret_cast<hipStream_t>(stream), seg,
                       coord, lsegs, nlong, nlong_dev, g, w, n, z, lo, alpha, beta, l1, l2);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

// long segments (lsegs: nlong segment ids), one wave each
int alink_ftrl_coord_long_f64(const int64_t* seg, const int64_t* coord, const int64_t* lsegs, int64_t nlong,
                              const int64_t* nlong_dev, const double* g, double* w, double* n, double* z, int64_t lo,
                              double alpha, double beta, double l1, double l2, int grid, void* stream) {
    if (nlong <= 0) return 0;
    if (alpha <= 0.0) return 1;
    const unsigned gb = nlong_dev != nullptr ? (unsigned)(grid > 0 ? grid : 1) : (unsigned)nlong;
    hipLaunchKernelGGL(ftrl_coord_long_kernel, dim3(gb), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), seg,
                       coord, lsegs, nlong, nlong_dev, g, w, n, z, lo, alpha, beta, l1, l2);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

int alink_ftrl_prox_f64(const int32_t* coords, int64_t m, double* w, const double* n, const double* z, double alpha,
                        double beta, double l1, double l2, int grid, void* stream) {
    if (m <= 0) return 0;
    if (grid <= 0 || alpha <= 0.0) return 1;
    hipLaunchKernelGGL(ftrl_prox_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), coords, m, w,
                       n, z, alpha, beta, l1, l2);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // extern "C"
