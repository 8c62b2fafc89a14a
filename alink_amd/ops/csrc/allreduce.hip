// One-shot all-reduce over IPC-mapped peer buffers — gfx950 / MI355X, xGMI.
//
// Reference semantics: AllReduce.java (A/common/comqueue/communication/AllReduce.java:85-120,192-360) — every
// task's buffer is cut into slices, slice owners sum them and the sums are broadcast back (reduce-scatter +
// all-gather over Flink's network).  For the small buffers of the BSP loop (KMeans [k][d+1] sums ~100 KB, loss
// and criterion scalars) the latency of a ring all-reduce dominates; on an xGMI-connected node every GPU can
// read every peer's memory directly, so the whole reduction is ONE kernel:
//
//   1. workgroup b copies slice b of the local input into this rank's staging slot (seq & 1) — double-buffered,
//      so a slot is rewritten only after every peer has finished reading it (they signalled the next call);
//   2. it releases (system scope) seq into flag[b][rank] of EVERY peer's flag array;
//   3. it spins (bounded by a real-time deadline) until flag[b][p] >= seq (mod 2^32) for all p in its own array;
//   4. it reads slice b of all P staging slots over xGMI and sums them in rank order 0..P-1 — the same order
//      on every rank, so all ranks hold bit-identical results (the determinism RCCL does not promise).
//
// Staging and flag memory are uncached device allocations (shared through hipIpcGetMemHandle), so remote
// writes and polls never see stale cache lines.  A peer that never arrives makes the kernel give up after a bounded number of polls, set
// *err and write NaN instead of hanging the job.  `phases` (bit 1: copy+signal, bit 2: wait+sum) lets a
// single-GPU test drive P virtual ranks one phase at a time.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstring>

namespace {

constexpr int TB = 256;

template <typename T, int OP>
__device__ __forceinline__ T combine(T a, T b) {
    if (OP == 0) return a + b;
    if (OP == 1) return b > a || b != b ? b : a;
    return b < a || b != b ? b : a;
}

// sum slice [lo, hi) of the P staging slots in rank order.  PP > 0: P is a compile-time constant, so the P remote
// loads of an element are all in flight before the first add (one xGMI round trip per element instead of P);
// PP == 0: runtime P (P > 8).
template <typename T, int OP, int PP>
__device__ __forceinline__ void sum_slots(char* const* __restrict__ peer_data, int P, int64_t slot_off, int64_t lo,
                                          int64_t hi, bool bad, T* out) {
    const int tid = threadIdx.x;
    if constexpr (PP > 0) {
        const T* src[PP];
#pragma unroll
        for (int p = 0; p < PP; ++p) src[p] = reinterpret_cast<const T*>(peer_data[p] + slot_off);
        for (int64_t i = lo + tid; i < hi; i += TB) {
            T v[PP];
#pragma unroll
            for (int p = 0; p < PP; ++p) v[p] = src[p][i];
            T acc = v[0];
#pragma unroll
            for (int p = 1; p < PP; ++p) acc = combine<T, OP>(acc, v[p]);
            out[i] = bad ? (T)__builtin_nan("") : acc;
        }
    } else {
        for (int64_t i = lo + tid; i < hi; i += TB) {
            T acc = reinterpret_cast<const T*>(peer_data[0] + slot_off)[i];
            for (int p = 1; p < P; ++p) acc = combine<T, OP>(acc, reinterpret_cast<const T*>(peer_data[p] + slot_off)[i]);
            out[i] = bad ? (T)__builtin_nan("") : acc;
        }
    }
}

template <typename T, int OP, int PP>
__global__ __launch_bounds__(TB) void oneshot_kernel(const T* in, T* out, int64_t n,
                                                     int P, int rank, uint32_t seq, char* const* __restrict__ peer_data,
                                                     uint32_t* const* __restrict__ peer_flags, int64_t slot_bytes,
                                                     int phases, uint64_t deadline_spins, int* __restrict__ err,
                                                     int* __restrict__ host_err) {
    const int tid = threadIdx.x;
    const int b = blockIdx.x;
    const int nb = gridDim.x;
    const int64_t per = (n + nb - 1) / nb;
    const int64_t lo = (int64_t)b * per;
    const int64_t hi = lo + per < n ? lo + per : n;
    const int64_t slot_off = (int64_t)(seq & 1u) * slot_bytes;
    if (phases & 1) {
        T* mine = reinterpret_cast<T*>(peer_data[rank] + slot_off);
        for (int64_t i = lo + tid; i < hi; i += TB) mine[i] = in[i];
        __threadfence_system();
        __syncthreads();
        if (tid < P)
            __hip_atomic_store(peer_flags[tid] + (int64_t)b * P + rank, seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (phases & 2) {
        if (tid < P) {
            const uint32_t* f = peer_flags[rank] + (int64_t)b * P + tid;
            uint64_t spins = 0;
            // wrap-safe: a peer may already have finished call seq and signalled seq + 1 before this wave's
            // first poll (a preempted wave, ranks time-sharing a GPU); any flag at or past seq means "arrived"
            // back-off: ~4096 short polls (~0.4 ms) at full rate, then s_sleep 64 (32x as long, counted as 32
            // spins so the deadline stays in time units) -- a late peer (ranks time-sharing one GPU, a rank still
            // in its compute kernel) no longer has the waiting waves take issue slots from its work
            while ((int32_t)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
                if (spins > deadline_spins) {
                    atomicOr(err, 1);
                    if (host_err != nullptr)          // mapped host word: the host sees the failure without a copy
                        __hip_atomic_store(host_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                if (spins < 4096) {
                    __builtin_amdgcn_s_sleep(2);
                    spins += 1;
                } else {
                    __builtin_amdgcn_s_sleep(64);
                    spins += 32;
                }
            }
        }
        __syncthreads();
        __threadfence_system();
        const bool bad = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        sum_slots<T, OP, PP>(peer_data, P, slot_off, lo, hi, bad, out);
    }
}

template <typename T, int OP, int PP>
void launch_p(const T* i, T* o, int64_t n, int P, int rank, uint32_t seq, char* const* pd, uint32_t* const* pf,
              int64_t slot_bytes, int blocks, int phases, uint64_t deadline, int* err, int* herr, hipStream_t st) {
    hipLaunchKernelGGL((oneshot_kernel<T, OP, PP>), dim3(blocks), dim3(TB), 0, st, i, o, n, P, rank, seq, pd, pf,
                       slot_bytes, phases, deadline, err, herr);
}

template <typename T, int OP>
void launch_op(const T* i, T* o, int64_t n, int P, int rank, uint32_t seq, char* const* pd, uint32_t* const* pf,
               int64_t slot_bytes, int blocks, int phases, uint64_t deadline, int* err, int* herr, hipStream_t st) {
    switch (P) {
        case 1: launch_p<T, OP, 1>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 2: launch_p<T, OP, 2>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 3: launch_p<T, OP, 3>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 4: launch_p<T, OP, 4>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 5: launch_p<T, OP, 5>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 6: launch_p<T, OP, 6>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 7: launch_p<T, OP, 7>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 8: launch_p<T, OP, 8>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        default: launch_p<T, OP, 0>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
    }
}

template <typename T>
int launch(int op, const void* in, void* out, int64_t n, int P, int rank, uint32_t seq, char* const* pd,
           uint32_t* const* pf, int64_t slot_bytes, int blocks, int phases, uint64_t deadline, int* err, int* herr,
           hipStream_t st) {
    const T* i = reinterpret_cast<const T*>(in);
    T* o = reinterpret_cast<T*>(out);
    switch (op) {
        case 0: launch_op<T, 0>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 1: launch_op<T, 1>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        case 2: launch_op<T, 2>(i, o, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, herr, st); break;
        default: return -2;
    }
    return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// Uncached device allocation (staging slots + flags), shareable with alink_ar_ipc_handle.
int alink_ar_alloc(int64_t bytes, void** out) {
    hipError_t e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached);
    if (e != hipSuccess) return (int)e;
    return (int)hipMemset(*out, 0, (size_t)bytes);
}

int alink_ar_free(void* p) { return (int)hipFree(p); }

// 64-byte IPC handle of an allocation made by alink_ar_alloc.
int alink_ar_ipc_handle(void* p, void* handle_out) {
    hipIpcMemHandle_t h;
    hipError_t e = hipIpcGetMemHandle(&h, p);
    if (e != hipSuccess) return (int)e;
    memcpy(handle_out, &h, sizeof(h));
    return 0;
}

int alink_ar_ipc_open(const void* handle, void** out) {
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

int alink_ar_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

int alink_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// one zeroed 64-byte line of mapped, coherent pinned host memory: *host = host address, *dev = kernel address
int alink_ar_host_word_alloc(void** host, void** dev) {
    hipError_t e = hipHostMalloc(host, 64, hipHostMallocMapped);
    if (e != hipSuccess) return (int)e;
    memset(*host, 0, 64);
    return (int)hipHostGetDevicePointer(dev, *host, 0);
}

int alink_ar_host_word_free(void* host) { return (int)hipHostFree(host); }

// peer_data / peer_flags: device arrays of P pointers (this rank's own entries included).
// dtype 0 f32, 1 f64; op 0 sum, 1 max, 2 min.
// in == out is allowed (in-place).  host_err (nullable): device address of a mapped host word that a timed-out
// call also sets (alink_ar_host_word_alloc), so the host can poll for failures without copying err back.
int alink_oneshot_allreduce(const void* in, void* out, int64_t n, int dtype, int op, int P, int rank, uint32_t seq,
                            void* const* peer_data, void* const* peer_flags, int64_t slot_bytes, int blocks,
                            int phases, double timeout_s, int* err, int* host_err, void* stream) {
    if (n <= 0) return 0;
    if (P < 1 || rank < 0 || rank >= P || blocks < 1 || blocks > 1024 || P > TB) return -1;
    const int64_t esz = dtype == 0 ? 4 : 8;
    if (n * esz > slot_bytes) return -3;
    // bounded poll: one s_sleep 2 (~128 clocks) + a system-scope load per spin, ~1e7 spins per second
    const uint64_t deadline = (uint64_t)(timeout_s * 1.0e7) + 1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    char* const* pd = reinterpret_cast<char* const*>(peer_data);
    uint32_t* const* pf = reinterpret_cast<uint32_t* const*>(peer_flags);
    if (dtype == 0)
        return launch<float>(op, in, out, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, host_err, st);
    if (dtype == 1)
        return launch<double>(op, in, out, n, P, rank, seq, pd, pf, slot_bytes, blocks, phases, deadline, err, host_err, st);
    return -2;
}

}  // extern "C"
