// Word2Vec skip-gram + hierarchical softmax, Hogwild on the GPU — gfx950 / MI355X.
//
// Reference: Word2VecTrainBatchOp.CalcModel (A/operator/batch/nlp/Word2VecTrainBatchOp.java:~425-505): for every
// centre position i with a random window shrink b, every context word x of the window trains its input vector
// h = syn0[x] against the Huffman path of the centre word: f = h . syn1[node], skip |f| >= 6, g = (1 - code -
// sigma(f)) * alpha from the 1/84-step sigmoid table, neu1e += g syn1[node], syn1[node] += g h; then syn0[x] +=
// neu1e.  One Java thread runs that loop per worker.
//
// Here one wave owns one centre position (the window enumeration happens on the device: no pair list is built
// on the host), lanes hold DPL = ceil(d/64) dimensions each, dots are wave reductions, and waves update the
// shared syn0 / syn1 tables without locks — the Hogwild scheme of the original word2vec.c threads.  With
// max_waves = 1 the launch is one wave and reproduces the sequential reference order exactly (tests).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

template <int DPL>
__global__ __launch_bounds__(256) void w2v_sg_hs_kernel(const int* __restrict__ tok, const int* __restrict__ dstart,
                                                        const int* __restrict__ dend, const int* __restrict__ shrink,
                                                        int64_t ntok, int window, const int8_t* __restrict__ codes,
                                                        const int* __restrict__ points, const int* __restrict__ lens,
                                                        int Lmax, float* __restrict__ syn0, float* __restrict__ syn1,
                                                        int d, float alpha) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wid; i < ntok; i += nw) {
        const int word = tok[i];
        const int b = shrink[i];
        const int L = lens[word];
        const int8_t* cd = codes + (int64_t)word * Lmax;
        const int* pt = points + (int64_t)word * Lmax;
        for (int a = b; a < 2 * window + 1 - b; ++a) {
            if (a == window) continue;
            const int64_t c = i - window + a;
            if (c < dstart[i] || c >= dend[i]) continue;
            const int x = tok[c];
            float* hx = syn0 + (int64_t)x * d;
            float h[DPL], e[DPL];
#pragma unroll
            for (int q = 0; q < DPL; ++q) {
                const int dd = lane + 64 * q;
                h[q] = dd < d ? hx[dd] : 0.f;
                e[q] = 0.f;
            }
            for (int l = 0; l < L; ++l) {
                float* o = syn1 + (int64_t)pt[l] * d;
                float ov[DPL];
                float part = 0.f;
#pragma unroll
                for (int q = 0; q < DPL; ++q) {
                    const int dd = lane + 64 * q;
                    ov[q] = dd < d ? o[dd] : 0.f;
                    part += ov[q] * h[q];
                }
                const float f = wave_sum(part);
                if (!(f > -6.0f && f < 6.0f)) continue;
                // sigmoid table abscissa: floor((f + 6) * 84) / 84 - 6  (EXP_TABLE_SIZE 1000 over [-6, 6))
                const float qf = floorf((f + 6.0f) * 84.0f) / 84.0f - 6.0f;
                const float sig = 1.0f / (1.0f + expf(-qf));
                const float g = (1.0f - (float)cd[l] - sig) * alpha;
#pragma unroll
                for (int q = 0; q < DPL; ++q) {
                    const int dd = lane + 64 * q;
                    e[q] += g * ov[q];
                    if (dd < d) o[dd] = ov[q] + g * h[q];
                }
            }
#pragma unroll
            for (int q = 0; q < DPL; ++q) {
                const int dd = lane + 64 * q;
                if (dd < d) hx[dd] = h[q] + e[q];
            }
        }
    }
}

}  // namespace

extern "C" {

// tok[ntok] vocabulary ids of the concatenated documents, dstart/dend[ntok] the bounds of each token's document,
// shrink[ntok] the random window shrink b; codes int8 / points int32 [V][Lmax], lens[V]; syn0 [V][d], syn1
// [V-1][d] fp32 updated in place.  max_waves > 0 caps the number of concurrent waves (1 = sequential order).
int alink_w2v_sg_hs_f32(const int* tok, const int* dstart, const int* dend, const int* shrink, int64_t ntok,
                        int window, const int8_t* codes, const int* points, const int* lens, int Lmax, float* syn0,
                        float* syn1, int d, float alpha, int max_waves, void* stream) {
    if (ntok <= 0) return 0;
    if (d < 1 || d > 512 || window < 1) return -1;
    int64_t waves = ntok < 65536 ? ntok : 65536;
    if (max_waves > 0 && waves > max_waves) waves = max_waves;
    const int block = waves >= 4 ? 256 : 64 * (int)waves;
    const int grid = (int)((waves * 64 + block - 1) / block);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int dpl = (d + 63) / 64;
#define W2V_LAUNCH(N) hipLaunchKernelGGL(w2v_sg_hs_kernel<N>, dim3(grid), dim3(block), 0, st, tok, dstart, dend, \
                                         shrink, ntok, window, codes, points, lens, Lmax, syn0, syn1, d, alpha)
    if (dpl == 1) W2V_LAUNCH(1);
    else if (dpl == 2) W2V_LAUNCH(2);
    else if (dpl <= 4) W2V_LAUNCH(4);
    else W2V_LAUNCH(8);
#undef W2V_LAUNCH
    return (int)hipGetLastError();
}

}  // extern "C"
