"""KMeans hot path: fused distance + argmin + per-cluster accumulation (kernels K1+K2).

``assign_accumulate(X, C)`` returns the ``[k, d+1]`` float64 buffer ``[sum_x | count]`` per centroid — the
``centroidAllReduce`` buffer of the reference (``KMeansAssignCluster.java:48-63``,
``KMeansUtil.updateSumMatrix`` ``KMeansUtil.java:60-85``) — for this rank's rows, ready for the BSP
all-reduce.

* GPU, bf16 rows, d == 128, k <= 128, unweighted: one persistent fused kernel + an fp64 fixed-order slab
  reduction (``csrc/kmeans_common.hip``, deterministic): ``csrc/kmeans_v10.hip`` for k <= 112 (the production
  kernel: MFMA distances, register-resident VALU accumulate; ``kernel_version``), ``csrc/kmeans_v7.hip`` for
  112 < k <= 128 (MFMA distances + one-hot MFMA accumulate).
* GPU, bf16 rows, d in {64, 128, 256}, k <= 256 (512 at d = 64), optionally weighted: two passes — the MFMA
  nearest-centroid kernel (``csrc/kmeans_nearest.hip``) then accumulate-by-index (``csrc/kmeans_accum.hip``:
  the MFMA one-hot GEMM for unweighted d = 128, LDS float atomics otherwise), with a fixed-order fp64 reduction.
* GPU, fp32 rows, d = 64 or a multiple of 128 up to 1024, k <= 256 (512 at d = 64), optionally weighted: the
  nearest centroid from a chunked fp32 GEMM (hipBLASLt) + argmax, then the accumulate-by-index kernel over the
  fp32 rows (``csrc/kmeans_accum.hip`` ``alink_kmeans_accum_f32``: fp64 LDS table, fixed-order fp64 reduction).
  fp64 feature matrices (VectorAssembler output) reach it through ``ALINK_KMEANS_INPUT=fp32`` (a one-time cast,
  see ``models/clustering/kmeans.train_kmeans``; ``bf16`` selects the fused bf16 kernels instead).
* anything else: chunked PyTorch path (fp64 on CPU; on GPU fp32 GEMM of the same bf16-rounded centroids).
"""
from __future__ import annotations

import os
import weakref
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib

__all__ = ["assign_accumulate", "assign", "assign_accumulate_torch", "hip_supported", "prepare_centroids",
           "general_supported", "assign_accumulate_general_hip", "accumulate_by_index_hip", "f32_supported",
           "assign_accumulate_f32_hip", "assign_f32"]

_BUF: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}
HIP_CALLS = 0  # launches of the fused HIP assign+accumulate path (bench / tests read it)
HIP_D = 128
HIP_KMAX = 128


def hip_supported(X: torch.Tensor, k: int) -> bool:
    return (X.is_cuda and X.dtype == torch.bfloat16 and X.dim() == 2 and X.shape[1] == HIP_D
            and 1 <= k <= HIP_KMAX and X.shape[0] > 0 and X.is_contiguous() and X.data_ptr() % 16 == 0)


_PREP = {}


_PREPARED = {}    # device -> (weakref to the centroid tensor whose operands sit in _PREP[device], its _version)


def _ckey(C: torch.Tensor):
    """Identity of a centroid tensor that cannot alias: a weak reference to the tensor owning the memory
    (compared by object identity; views resolve to their base) plus (data_ptr, shape, version).  The address
    alone could match a fresh tensor that the caching allocator placed where a freed one was — e.g. the next
    KMeans job's initial centroids."""
    base = C if C._base is None else C._base
    return (weakref.ref(base), C.data_ptr(), tuple(C.shape), C._version)


def key_matches(key, C: torch.Tensor) -> bool:
    if key is None:
        return False
    base = C if C._base is None else C._base
    return key[0]() is base and key[1:] == (C.data_ptr(), tuple(C.shape), C._version)


def _prepared_is(dev_index, C: torch.Tensor) -> bool:
    return key_matches(_PREPARED.get(dev_index), C)


def prepare_centroids(C: torch.Tensor, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Padded bf16 centroid block [128,128] and accumulator init -|c|^2/2 (of the bf16-rounded centroids).
    fp64 centroids on the GPU go through one HIP launch into per-device buffers (stream-ordered reuse); when
    ``update_centroids_hip`` already wrote the operands of exactly this tensor, nothing is launched."""
    k = C.shape[0]
    if C.is_cuda and C.dtype == torch.float64 and C.shape[1] == HIP_D and k <= HIP_KMAX:
        if _prepared_is(C.device.index, C) and C.device.index in _PREP:
            return _PREP[C.device.index]
        L = _lib.require()
        key = C.device.index
        if key not in _PREP:
            _PREP[key] = (torch.empty((HIP_KMAX, HIP_D), dtype=torch.bfloat16, device=C.device),
                          torch.empty((HIP_KMAX,), dtype=torch.float32, device=C.device))
        cpad, ninit = _PREP[key]
        Cc = C.contiguous()
        rc = L.alink_kmeans_prep_centroids(Cc.data_ptr(), k, cpad.data_ptr(), ninit.data_ptr(), _lib.stream_ptr(C.device))
        if rc != 0:
            raise RuntimeError(f"alink_kmeans_prep_centroids failed: {rc}")
        _PREPARED[key] = _ckey(C) if Cc is C else None
        return cpad, ninit
    cb = C.to(device=device, dtype=torch.bfloat16)
    cpad = torch.zeros((HIP_KMAX, HIP_D), dtype=torch.bfloat16, device=device)
    cpad[:k] = cb
    ninit = torch.full((HIP_KMAX,), -3.0e38, dtype=torch.float32, device=device)
    ninit[:k] = -0.5 * (cb.float() ** 2).sum(1)
    return cpad, ninit


KERNEL_VERSIONS = ("v7", "v10")
# v7 variant (csrc/kmeans_v7.hip VAR): 0 = all 8 waves stage the tile ring; 1 (default) = the accumulate waves
# stage it all, so the distance waves (the critical role) carry no LDS-DMA issue cost or vmcnt waits
V7_VAR = int(os.environ.get("ALINK_KMEANS_V7_VAR", "1"))
# v10 launch flags (csrc/kmeans_v10.hip mode bit 4): 1 (default) = default-policy X loads, 0 = non-temporal.
# Under the full kernel the default policy measured 2-5 % faster on every box (profiles/kmeans_v10_r3.txt),
# although the load pipeline alone streams faster with nt
V10_FLAGS = int(os.environ.get("ALINK_KMEANS_V10_FLAGS", "1"))
V10_KMAX = 112
# serpentine tile order across Lloyd supersteps (serpentine_reverse)
SERPENTINE = os.environ.get("ALINK_KMEANS_SERPENTINE", "1") != "0"
# v10 work-stealing tail (csrc/kmeans_v10.hip DYN), opt-in: the last V10_POOL of the tiles are claimed at run time
# so workgroups on a slower XCD take fewer of them.  Measured (profiles/kmeans_dyn_r5.txt): the workgroups' exits
# line up (spread 40-190 us -> ~12 us) but the per-tile cost of the dynamic indexing makes the launch ~4 % slower,
# and which workgroup sums which rows (fp32) then varies run to run — so the deterministic static split (0) stays
# the default
V10_POOL = float(os.environ.get("ALINK_KMEANS_V10_POOL", "0"))
_DYN: Dict[int, list] = {}        # device -> [two int32 counters, launch parity]


def kernel_version(k: int = 100) -> str:
    """Fused assign+accumulate kernel for k centroids: v10 (csrc/kmeans_v10.hip: MFMA distances + register
    accumulate) for k <= 112, v7 (csrc/kmeans_v7.hip: one-hot MFMA accumulate) above.  ``ALINK_KMEANS_KERNEL``
    forces one (v10 only where k <= 112)."""
    v = os.environ.get("ALINK_KMEANS_KERNEL")
    if v is not None and v not in KERNEL_VERSIONS:
        raise ValueError(f"ALINK_KMEANS_KERNEL must be one of {KERNEL_VERSIONS}")
    if v is None:
        v = "v10" if k <= V10_KMAX else "v7"
    if v == "v10" and k > V10_KMAX:
        v = "v7"
    return v


_CUS: Dict[int, int] = {}
_GRID: Dict[Tuple, int] = {}

# per-rank assign time (bench.py's straggler split): while on, every assign+accumulate call is bracketed by HIP
# events on the caller's stream (GPU) or timed on the host (CPU paths)
_KT = {"on": False, "ev": [], "host_s": 0.0, "n": 0}


def kernel_timing(on: bool) -> None:
    """Start / stop recording the device time of every assign+accumulate call (events are collected later)."""
    _KT["on"] = bool(on)


def kernel_timing_collect() -> Tuple[int, float]:
    """(calls, seconds) of the assign+accumulate work recorded since the last collect (synchronises the events)."""
    n, sec = _KT["n"], _KT["host_s"]
    for a, b in _KT["ev"]:
        b.synchronize()
        sec += a.elapsed_time(b) * 1e-3
    _KT.update(ev=[], host_s=0.0, n=0)
    return n, sec


class _timed:
    """Bracket one assign+accumulate call when ``kernel_timing`` is on (no-op otherwise)."""
    __slots__ = ("dev", "e0", "t0")

    def __init__(self, dev):
        self.dev = dev if _KT["on"] else None

    def __enter__(self):
        if self.dev is not None:
            if self.dev.type == "cuda":
                self.e0 = torch.cuda.Event(enable_timing=True)
                self.e0.record(torch.cuda.current_stream(self.dev))
            else:
                import time
                self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.dev is not None:
            _KT["n"] += 1
            if self.dev.type == "cuda":
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(torch.cuda.current_stream(self.dev))
                _KT["ev"].append((self.e0, e1))
            else:
                import time
                _KT["host_s"] += time.perf_counter() - self.t0
        return False


def _num_cus(device) -> int:
    idx = torch.device(device).index or 0
    if idx not in _CUS:
        _CUS[idx] = torch.cuda.get_device_properties(device).multi_processor_count
    return _CUS[idx]


def assign_accumulate_hip(X: torch.Tensor, C: torch.Tensor, grid: Optional[int] = None,
                          assign_out: Optional[torch.Tensor] = None, mode: int = 0,
                          reverse: bool = False, skip: Optional[torch.Tensor] = None) -> torch.Tensor:
    with _timed(X.device):
        return _assign_accumulate_hip(X, C, grid, assign_out, mode, reverse, skip)


def _assign_accumulate_hip(X: torch.Tensor, C: torch.Tensor, grid: Optional[int] = None,
                           assign_out: Optional[torch.Tensor] = None, mode: int = 0,
                           reverse: bool = False, skip: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[k, d+1] fp64 sums|counts of this rank's rows (``csrc/kmeans_v10.hip`` for k <= 112, else
    ``csrc/kmeans_v7.hip``: role-split waves on 16x16x32 MFMA, LDS-DMA tile ring; ``kernel_version``).
    ``assign_out`` (int32 [N]) also receives every row's centroid id; ``mode`` 1/2 are the kernel's load-only /
    compute-only diagnostics (results meaningless).  ``reverse`` (v10): every workgroup walks its rows backwards —
    Lloyd alternates it per superstep (serpentine order), so a pass starts on the rows the previous pass read last,
    which are still in the Infinity Cache.  Same assignments and counts; the fp32 sums differ only in order.
    ``skip`` (v10, static split): a device word written by ``update_centroids_hip(..., skip_tol=)``; when it is
    nonzero at run time the launch returns at once and the result is garbage (the caller drops it)."""
    global HIP_CALLS
    L = _lib.require()
    HIP_CALLS += 1
    dev = X.device
    k = C.shape[0]
    if not hip_supported(X, k):
        raise ValueError("HIP KMeans path needs contiguous bf16 [N,128] on GPU and k <= 128")
    if assign_out is not None and (assign_out.dtype != torch.int32 or assign_out.numel() < X.shape[0]
                                   or assign_out.device != dev or not assign_out.is_contiguous()):
        raise ValueError("assign_out must be a contiguous int32 [N] tensor on X's device")
    cpad, ninit = prepare_centroids(C, dev)
    n = X.shape[0]
    ver = kernel_version(k)
    gkey = (ver, n, grid, dev.index)
    if gkey not in _GRID:      # per-shape launch geometry (one ctypes call per shape, not per superstep)
        _GRID[gkey] = int(getattr(L, f"alink_kmeans_{ver}_grid")(n, grid if grid is not None else _num_cus(dev)))
    grid = _GRID[gkey]
    key = (dev.index, grid)
    if key not in _BUF:
        # zeroed once: the kernels write only the first 16*ceil(k/16) rows of a slab, so the tail would otherwise
        # hold whatever the allocator recycled (NaN bit patterns included)
        _BUF[key] = (torch.zeros((grid, HIP_KMAX, HIP_D), dtype=torch.float32, device=dev),
                     torch.zeros((grid, HIP_KMAX), dtype=torch.float32, device=dev))
    slab, slab_cnt = _BUF[key]
    out = torch.empty((k, HIP_D + 1), dtype=torch.float64, device=dev)
    st = _lib.stream_ptr(dev)
    if mode < 16:
        mode |= (V7_VAR << 4) if ver == "v7" else (V10_FLAGS << 4)
    if reverse and ver == "v10":
        mode |= 32
    skipped = skip is not None and ver == "v10" and V10_POOL <= 0
    if skipped:
        rc = L.alink_kmeans_assign_accum_bf16_v10s(
            X.data_ptr(), n, cpad.data_ptr(), ninit.data_ptr(), k, slab.data_ptr(), slab_cnt.data_ptr(), grid, st,
            None if assign_out is None else assign_out.data_ptr(), int(mode), skip.data_ptr())
    elif ver == "v10" and V10_POOL > 0 and (mode & 7) == 0 and hasattr(L, "alink_kmeans_assign_accum_bf16_v10d"):
        dyn = _DYN.get(dev.index)
        if dyn is None:
            dyn = _DYN[dev.index] = [torch.zeros(2, dtype=torch.int32, device=dev), 0]
        rc = L.alink_kmeans_assign_accum_bf16_v10d(
            X.data_ptr(), n, cpad.data_ptr(), ninit.data_ptr(), k, slab.data_ptr(), slab_cnt.data_ptr(), grid, st,
            None if assign_out is None else assign_out.data_ptr(), int(mode), dyn[0].data_ptr(), dyn[1], V10_POOL)
        dyn[1] ^= 1
    else:
        rc = getattr(L, f"alink_kmeans_assign_accum_bf16_{ver}")(
            X.data_ptr(), n, cpad.data_ptr(), ninit.data_ptr(), k, slab.data_ptr(), slab_cnt.data_ptr(), grid, st,
            None if assign_out is None else assign_out.data_ptr(), int(mode))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_assign_accum_bf16_{ver} failed: {rc}")
    if skipped and hasattr(L, "alink_kmeans_reduce_slabs2"):
        # the reduction reads the same skip word: a skipped launch costs two empty kernels, not a slab pass
        rc = L.alink_kmeans_reduce_slabs2(slab.data_ptr(), slab_cnt.data_ptr(), grid, k, out.data_ptr(),
                                          skip.data_ptr(), st)
    else:
        rc = L.alink_kmeans_reduce_slabs(slab.data_ptr(), slab_cnt.data_ptr(), grid, k, out.data_ptr(), st)
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_reduce_slabs failed: {rc}")
    return out


_STAT = {}
# wait for the update's stats by polling a sequence word in the mapped memory instead of a stream event: no event
# marker between the update and the speculative next-superstep launch (a ~6 us launch gap per superstep,
# profiles/gpu_tests_r5.txt); ALINK_KMEANS_HOST_POLL=0 waits on an event
HOST_POLL = os.environ.get("ALINK_KMEANS_HOST_POLL", "1") != "0"
HOST_POLL_TIMEOUT_S = 120.0
_SKIP = {}      # device -> int32 [1] skip word of the last update (empty cluster or converged; speculative launches read it)


class _HostStat:
    """Per-device result words of the fused update: ``stat`` (3 device u64: max-shift bits, empty flag, the
    kernel's completion ticket; all-zero between launches) and 16 bytes of mapped pinned host memory that the
    kernel's last block writes directly, so a superstep needs neither a memset before the update nor a
    device->host copy after it.  If mapped host memory cannot be had, the update falls back to memset + copy."""

    def __init__(self, L, dev):
        import ctypes
        self.stat = torch.zeros(3, dtype=torch.int64, device=dev)
        self.host, self.dev_ptr, self._view = None, None, None
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        if os.environ.get("ALINK_KMEANS_HOST_STAT", "1") != "0" and \
                L.alink_kmeans_host_stat_alloc(ctypes.byref(h), ctypes.byref(d)) == 0 and d.value:
            self._hptr, self.dev_ptr = h.value, d.value
            self._view = np.ctypeslib.as_array((ctypes.c_uint64 * 3).from_address(h.value))
            self._L = L
        else:
            self.host = torch.empty(2, dtype=torch.int64, pin_memory=True)
        self.seq = 0

    def next_seq(self) -> int:
        """Sequence number of the next update launch (0: no host poll -- the caller waits on an event)."""
        if self._view is None or not HOST_POLL:
            return 0
        self.seq += 1
        return self.seq

    def wait(self, seq: int, dev) -> None:
        """Until the update launched with ``seq`` has published its stats (a tight poll of the mapped word, then
        20 us sleeps); past ``HOST_POLL_TIMEOUT_S`` the stream is synchronised and the word must be there."""
        view = self._view
        for _ in range(4000):
            if int(view[2]) == seq:
                return
        import time
        t_end = time.perf_counter() + HOST_POLL_TIMEOUT_S
        while time.perf_counter() < t_end:
            if int(view[2]) == seq:
                return
            time.sleep(20e-6)
        torch.cuda.current_stream(dev).synchronize()
        if int(view[2]) != seq:
            raise RuntimeError(f"kmeans_update completed without publishing sequence {seq}")

    def values(self):
        if self._view is not None:
            return int(self._view[0]), int(self._view[1])
        return int(self.host[0]), int(self.host[1])

    def __del__(self):
        try:
            if self._view is not None:
                self._view = None
                self._L.alink_kmeans_host_stat_free(self._hptr)
        except Exception:
            pass


def update_supported(buf: torch.Tensor) -> bool:
    return buf.is_cuda and buf.dtype == torch.float64 and buf.dim() == 2 and buf.shape[1] == HIP_D + 1 and \
        1 <= buf.shape[0] <= HIP_KMAX and buf.is_contiguous()


def operand_hysteresis() -> bool:
    """bf16 centroid-operand hysteresis in the fused update (default on; ``ALINK_KMEANS_HYSTERESIS=0`` disables)."""
    return os.environ.get("ALINK_KMEANS_HYSTERESIS", "1") != "0"


def update_centroids_hip(buf: torch.Tensor, prev: Optional[torch.Tensor], deferred: bool = False,
                         hysteresis: Optional[bool] = None, skip_tol: Optional[float] = None):
    """Fused Lloyd update on the all-reduced ``[k, 129]`` buffer (``csrc/kmeans_common.hip``): returns
    ``(C [k,128] fp64, max_shift vs prev or None, any_empty)`` with ONE 16-byte device->host read, and leaves
    the next superstep's bf16 operands prepared (``prepare_centroids`` of the returned C launches nothing).
    ``deferred=True`` returns ``(C, read)`` instead: ``read()`` waits for the stats later, so the caller can queue
    more GPU work (the next superstep's assign kernel) first.  ``skip_tol`` (with ``deferred``): the kernel also
    writes a device word = (some cluster empty, or prev given and max shift < skip_tol) — ``read.skip`` is that word (None
    when unavailable), for a speculative ``assign_accumulate_hip(..., skip=read.skip)`` to return at once on
    convergence; the caller must drop such a result whenever ``shift < skip_tol`` or a cluster is empty."""
    L = _lib.require()
    dev = buf.device
    k = buf.shape[0]
    if dev.index not in _PREP:
        _PREP[dev.index] = (torch.empty((HIP_KMAX, HIP_D), dtype=torch.bfloat16, device=dev),
                            torch.empty((HIP_KMAX,), dtype=torch.float32, device=dev))
    if dev.index not in _STAT:
        _STAT[dev.index] = _HostStat(L, dev)
    hs = _STAT[dev.index]
    stat = hs.stat
    cpad, ninit = _PREP[dev.index]
    use_prev = prev is not None and prev.is_cuda and prev.dtype == torch.float64 and tuple(prev.shape) == (k, HIP_D)
    pv = prev.contiguous() if use_prev else None
    C = torch.empty((k, HIP_D), dtype=torch.float64, device=dev)
    if hysteresis is None:
        hysteresis = operand_hysteresis()
    skip = None
    if skip_tol is not None and hs.dev_ptr is not None:
        skip = _SKIP.get(dev.index)
        if skip is None:
            skip = _SKIP[dev.index] = torch.zeros(1, dtype=torch.int32, device=dev)
    seq = hs.next_seq()
    rc = L.alink_kmeans_update2(buf.data_ptr(), k, None if pv is None else pv.data_ptr(), C.data_ptr(),
                                cpad.data_ptr(), ninit.data_ptr(), stat.data_ptr(), int(bool(hysteresis)),
                                hs.dev_ptr, float(skip_tol) if skip is not None else 0.0,
                                None if skip is None else skip.data_ptr(), seq, _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_update failed: {rc}")
    if hs.dev_ptr is None:
        hs.host.copy_(stat[:2], non_blocking=True)
    ev = None
    if not seq:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
    _PREPARED[dev.index] = _ckey(C)

    def read():
        """Wait for THIS update's 16-byte stats only (work queued after it, e.g. a speculative next-step
        kernel, keeps running) and return (max_shift or None, any_empty)."""
        if seq:
            hs.wait(seq, dev)
        else:
            ev.synchronize()
        shift_bits, empty = hs.values()
        shift = float(np.frombuffer(np.int64(shift_bits).tobytes(), dtype=np.float64)[0]) if use_prev else None
        return shift, bool(empty)
    read.skip = skip
    if deferred:
        return C, read
    shift, empty = read()
    return C, shift, empty


COST1_GRID = int(os.environ.get("ALINK_KMEANS_COST1_GRID", "4"))    # streaming workgroups per CU (all resident)
COST1_VARIANT = int(os.environ.get("ALINK_KMEANS_COST1_VARIANT", "1"))  # csrc: rows in flight / load policy


def cost1_hip(X: torch.Tensor, c: torch.Tensor, with_sum: bool = False):
    """fp64 [N] Euclidean distance of every row of X to ONE center (rounded to bf16: k-means|| centers are rows of
    X) -- ``csrc/kmeans_nearest.hip`` kmeans_cost1_kernel, one coalesced streaming pass (the first k-means|| cost).
    ``with_sum``: also the per-wave sums of the costs (fp64 [waves], a fixed order for a given grid), so the
    oversampling threshold's total needs no second pass over the [N] costs: returns (cost, partial sums)."""
    L = _lib.require()
    if not nearest_supported(X):
        raise ValueError("cost1_hip needs contiguous bf16 [N, D] on GPU with D in (64, 128, 256)")
    n, d = X.shape
    cb = c.reshape(-1).to(device=X.device, dtype=torch.bfloat16).contiguous()
    if cb.numel() != d:
        raise ValueError("center shape mismatch")
    cost = torch.empty(n, dtype=torch.float64, device=X.device)
    grid = COST1_GRID * _num_cus(X.device)
    wsum = torch.empty(grid * 4, dtype=torch.float64, device=X.device) if with_sum else None
    rc = L.alink_kmeans_cost1_bf16_sum(X.data_ptr(), n, d, cb.data_ptr(), cost.data_ptr(),
                                       None if wsum is None else wsum.data_ptr(), grid, COST1_VARIANT,
                                       _lib.stream_ptr(X.device))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_cost1_bf16 failed: {rc}")
    return (cost, wsum) if with_sum else cost


def nearest_counts_hip(X: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    """int64 [m]: how many rows of X have each centroid as their nearest — ``nearest_hip`` + ``bincount`` in ONE
    pass with no per-row output (per-workgroup LDS counts, integer global adds) when the m <= 256 centroids fit one
    launch; otherwise the two-step form.  Ties and rounding exactly as ``nearest_hip``."""
    L = _lib.require()
    if not nearest_supported(X):
        raise ValueError("nearest_counts_hip needs contiguous bf16 [N, D] on GPU with D in (64, 128, 256)")
    n, d = X.shape
    m = C.shape[0]
    if m > NEAREST_CHUNK:
        return torch.bincount(nearest_hip(X, C)[0].to(torch.int64), minlength=m)
    Cb = C.to(device=X.device, dtype=torch.bfloat16).contiguous()
    if Cb.shape[1] != d or m == 0:
        raise ValueError("centroid shape mismatch")
    chalf = (0.5 * (Cb.float() ** 2).sum(1)).contiguous()
    counts = torch.zeros(m, dtype=torch.int64, device=X.device)
    rg = _rg(d, m)
    rc = L.alink_kmeans_nearest_bf16_rg(X.data_ptr(), n, d, Cb.data_ptr(), chalf.data_ptr(), m, 0, None, None, 0,
                                        NEAREST_GRID * _num_cus(X.device), rg, counts.data_ptr(),
                                        _lib.stream_ptr(X.device))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_nearest_bf16 (counts) failed: {rc}")
    return counts


def _scores(Xc: torch.Tensor, C: torch.Tensor, emulate_bf16: bool) -> torch.Tensor:
    """x.c - |c|^2/2 (argmax == argmin of squared euclidean distance)."""
    if emulate_bf16:
        cb = C.to(torch.bfloat16).float()
        return Xc.float() @ cb.T - 0.5 * (cb ** 2).sum(1)
    Cd = C.to(Xc.dtype)
    return Xc @ Cd.T - 0.5 * (Cd ** 2).sum(1)


def assign_accumulate_torch(X: torch.Tensor, C: torch.Tensor, weights: Optional[torch.Tensor] = None,
                            chunk: int = 1 << 20) -> torch.Tensor:
    """Reference implementation: [k, d+1] float64 sums/counts of the nearest-centroid assignment."""
    k, d = C.shape
    out = torch.zeros((k, d + 1), dtype=torch.float64, device=X.device)
    low = X.dtype in (torch.bfloat16, torch.float16)
    for s in range(0, X.shape[0], chunk):
        xc = X[s:s + chunk]
        if not low:
            xc = xc.to(torch.float64)
        idx = _scores(xc, C, low).argmax(1)
        w = None if weights is None else weights[s:s + chunk].to(torch.float64)
        xs = xc.to(torch.float64)
        if w is not None:
            xs = xs * w[:, None]
        out[:, :d].index_add_(0, idx, xs)
        out[:, d].index_add_(0, idx, torch.ones_like(idx, dtype=torch.float64) if w is None else w)
    return out


def general_supported(X: torch.Tensor, k: int) -> bool:
    """Shapes of the two-pass HIP path (nearest + accumulate-by-index)."""
    return nearest_supported(X) and 1 <= k <= (512 if X.shape[1] == 64 else 256)


GENERAL_CALLS = 0
_ACC: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}


def accumulate_by_index_hip(X: torch.Tensor, idx: torch.Tensor, k: int,
                            weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[k, d+1] fp64 ``[sum_r w_r x_r | sum_r w_r]`` per index value (``csrc/kmeans_accum.hip``)."""
    L = _lib.require()
    n, d = X.shape
    dev = X.device
    if idx.dtype != torch.int32 or idx.numel() != n or idx.device != dev:
        raise ValueError("idx must be int32 [N] on X's device")
    w = None
    if weights is not None:
        w = weights.to(device=dev, dtype=torch.float32).contiguous()
        if w.numel() != n:
            raise ValueError("weights length mismatch")
    if X.dtype == torch.float32:
        return _accumulate_f32(L, X, idx, k, w)
    if d == HIP_D // 2 and w is None and k <= 256 and X.is_contiguous() and n >= 2:
        # d = 64 on the d = 128 MFMA kernel: view row v = (row 2v | row 2v+1); pass A one-hot by idx[2v] keeps
        # dims 0..63, pass B by idx[2v+1] keeps dims 64..127 — two reads of X at MFMA speed instead of one pass of
        # LDS float atomics (an odd last row is added on the host side)
        m = n // 2
        Xv = X[:2 * m].view(m, HIP_D)
        outA = accumulate_by_index_hip(Xv, idx[0:2 * m:2].contiguous(), k)
        outB = accumulate_by_index_hip(Xv, idx[1:2 * m:2].contiguous(), k)
        out = torch.cat([outA[:, :d] + outB[:, d:HIP_D], outA[:, HIP_D:] + outB[:, HIP_D:]], 1)
        if n % 2:
            c = int(idx[n - 1].item())
            if 0 <= c < k:
                out[c, :d] += X[n - 1].to(torch.float64)
                out[c, d] += 1.0
        return out
    if d == 2 * HIP_D and w is None and k <= 128 and X.is_contiguous():
        # d = 256 on the d = 128 MFMA kernel: row r = view rows 2r (dims 0..127) and 2r+1 (dims 128..255), the
        # second half accumulated under virtual centroid c + k (same bytes read, one-hot GEMM of 2k rows)
        idx2 = torch.stack([idx, torch.where(idx >= 0, idx + k, idx)], 1).reshape(-1).contiguous()
        out2 = accumulate_by_index_hip(X.view(2 * n, HIP_D), idx2, 2 * k)
        return torch.cat([out2[:k, :HIP_D], out2[k:, :HIP_D], out2[:k, HIP_D:]], 1)
    if d == HIP_D and w is None and k <= 256:
        # MFMA one-hot GEMM fed by idx (csrc/kmeans_accum.hip kmeans_accum_mfma_kernel)
        grid = _num_cus(dev)
        key = (dev.index, grid, k, d, "mfma")
        if key not in _ACC:
            _ACC.clear()
            _ACC[key] = (torch.empty(grid * k * d, dtype=torch.float32, device=dev),
                         torch.empty(grid * k, dtype=torch.float32, device=dev))
        slab, slab_cnt = _ACC[key]
        out = torch.empty((k, d + 1), dtype=torch.float64, device=dev)
        rc = L.alink_kmeans_accum_mfma_bf16(X.data_ptr(), n, idx.contiguous().data_ptr(), k, grid, slab.data_ptr(),
                                            slab_cnt.data_ptr(), out.data_ptr(), _lib.stream_ptr(dev))
        if rc != 0:
            raise RuntimeError(f"alink_kmeans_accum_mfma_bf16 failed: {rc}")
        return out
    nchunk = max(1, min(_num_cus(dev), (n + 4095) // 4096))
    key = (dev.index, nchunk, k, d)
    if key not in _ACC:
        _ACC.clear()
        _ACC[key] = (torch.empty(nchunk * k * d, dtype=torch.float32, device=dev),
                     torch.empty(nchunk * k, dtype=torch.float32, device=dev))
    slab, slab_cnt = _ACC[key]
    out = torch.empty((k, d + 1), dtype=torch.float64, device=dev)
    rc = L.alink_kmeans_accum_bf16(X.data_ptr(), n, d, idx.contiguous().data_ptr(),
                                   None if w is None else w.data_ptr(), k, nchunk, slab.data_ptr(),
                                   slab_cnt.data_ptr(), out.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_accum_bf16 failed: {rc}")
    return out


def _accumulate_f32(L, X: torch.Tensor, idx: torch.Tensor, k: int, w: Optional[torch.Tensor]) -> torch.Tensor:
    n, d = X.shape
    dev = X.device
    if not f32_supported(X, k):
        raise ValueError("fp32 accumulate needs contiguous 16-B aligned fp32 [N, D] (D = 64 or a multiple of 128 "
                         "up to 1024) on the GPU and k within the LDS table limit")
    nchunk = max(1, min(_num_cus(dev), (n + 4095) // 4096))
    key = (dev.index, nchunk, k, d, "f32")
    if key not in _ACC:
        _ACC.clear()
        _ACC[key] = (torch.empty(nchunk * k * d, dtype=torch.float32, device=dev),
                     torch.empty(nchunk * k, dtype=torch.float32, device=dev))
    slab, slab_cnt = _ACC[key]
    out = torch.empty((k, d + 1), dtype=torch.float64, device=dev)
    rc = L.alink_kmeans_accum_f32(X.data_ptr(), n, d, idx.contiguous().data_ptr(), None if w is None else w.data_ptr(),
                                  k, nchunk, slab.data_ptr(), slab_cnt.data_ptr(), out.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_accum_f32 failed: {rc}")
    return out


def f32_supported(X: torch.Tensor, k: int) -> bool:
    """Shapes of the fp32 path (GEMM assignment + fp32 accumulate-by-index kernel)."""
    if not (X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and X.shape[0] > 0 and X.is_contiguous()
            and X.data_ptr() % 16 == 0):
        return False
    d = X.shape[1]
    return (d == 64 or (d % 128 == 0 and d <= 1024)) and 1 <= k <= (512 if d == 64 else 256)


F32_CALLS = 0


def assign_f32(X: torch.Tensor, C: torch.Tensor, chunk: int = 1 << 21) -> torch.Tensor:
    """int32 nearest-centroid index of every fp32 row: x.c - |c|^2/2 by an fp32 GEMM per chunk, argmax."""
    Cf = C.to(device=X.device, dtype=torch.float32)
    half = 0.5 * (Cf * Cf).sum(1)
    idx = torch.empty(X.shape[0], dtype=torch.int32, device=X.device)
    for s in range(0, X.shape[0], chunk):
        sc = torch.addmm(half.neg()[None, :], X[s:s + chunk], Cf.T)
        idx[s:s + chunk] = sc.argmax(1).to(torch.int32)
    return idx


def assign_accumulate_f32_hip(X: torch.Tensor, C: torch.Tensor,
                              weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[k, d+1] fp64 sums|counts over fp32 rows: ``assign_f32`` + the fp32 accumulate-by-index kernel."""
    global F32_CALLS
    F32_CALLS += 1
    return accumulate_by_index_hip(X, assign_f32(X, C), C.shape[0], weights)


_HELD: Dict[Tuple, torch.Tensor] = {}


def held_operand(C: torch.Tensor) -> torch.Tensor:
    """bf16 centroid operand with the same hysteresis as the fused update kernel (kmeans_common.hip): a coordinate
    keeps its previous operand while the fp64 centroid stays within one bf16 ulp of the row's largest coordinate,
    so Lloyd reaches an exactly stationary assignment instead of cycling on re-quantisation jitter."""
    Cb = C.to(torch.bfloat16)
    key = (C.device.index, tuple(C.shape))
    prev = _HELD.get(key)
    if prev is not None and operand_hysteresis():
        m = C.abs().amax(1, keepdim=True).float()
        band = torch.ldexp(torch.ones_like(m), torch.frexp(m)[1] - 8).double()
        keep = ((C.double() - prev.double()).abs() < band) & (m > 0)
        Cb = torch.where(keep, prev, Cb)
    if len(_HELD) > 8:
        _HELD.clear()
    _HELD[key] = Cb
    return Cb


def assign_accumulate_general_hip(X: torch.Tensor, C: torch.Tensor,
                                  weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Two-pass HIP path for the shapes v7 does not cover (d 64/256, k up to 256/512, weighted rows)."""
    global GENERAL_CALLS
    if not general_supported(X, C.shape[0]):
        raise ValueError("general HIP KMeans path needs contiguous bf16 [N, D in (64,128,256)] and k <= 256")
    GENERAL_CALLS += 1
    idx, _ = nearest_hip(X, held_operand(C) if C.dtype != torch.bfloat16 else C)
    return accumulate_by_index_hip(X, idx, C.shape[0], weights)


def serpentine_reverse(step: int) -> bool:
    """Lloyd's walk direction at superstep ``step`` (1-based): with ``ALINK_KMEANS_SERPENTINE`` on (default),
    even supersteps walk every workgroup's rows backwards (``assign_accumulate_hip(reverse=...)``).  A function of
    the step only, so a run is reproducible and a speculative next-step launch uses the direction of its step."""
    return SERPENTINE and step % 2 == 0


def assign_accumulate(X: torch.Tensor, C: torch.Tensor, weights: Optional[torch.Tensor] = None,
                      reverse: bool = False) -> torch.Tensor:
    hip_ok = _lib.available() or not _lib.torch_fallback_allowed()
    if weights is None and hip_supported(X, C.shape[0]) and hip_ok:
        return assign_accumulate_hip(X, C, reverse=reverse)
    with _timed(X.device):
        if general_supported(X, C.shape[0]) and hip_ok:
            return assign_accumulate_general_hip(X, C, weights)
        if f32_supported(X, C.shape[0]) and hip_ok:
            return assign_accumulate_f32_hip(X, C, weights)
        return assign_accumulate_torch(X, C, weights)


def assign(X: torch.Tensor, C: torch.Tensor, chunk: int = 1 << 20) -> Tuple[torch.Tensor, torch.Tensor]:
    """Nearest centroid index and squared euclidean distance for every row."""
    if nearest_supported(X) and (_lib.available() or not _lib.torch_fallback_allowed()):
        idx, d2 = nearest_hip(X, C)
        return idx.to(torch.int64), d2.to(torch.float64)
    low = X.dtype in (torch.bfloat16, torch.float16)
    idx_all, d2_all = [], []
    for s in range(0, X.shape[0], chunk):
        xc = X[s:s + chunk]
        if not low:
            xc = xc.to(torch.float64)
        sc = _scores(xc, C, low)
        best, idx = sc.max(1)
        xn = (xc.to(torch.float64) ** 2).sum(1)
        d2 = (xn - 2.0 * best.to(torch.float64)).clamp_min(0.0)
        idx_all.append(idx)
        d2_all.append(d2)
    if not idx_all:
        return (torch.zeros(0, dtype=torch.int64, device=X.device),
                torch.zeros(0, dtype=torch.float64, device=X.device))
    return torch.cat(idx_all), torch.cat(d2_all)


NEAREST_DIMS = (64, 128, 256)
NEAREST_CHUNK = 256
# 32-row groups per wave iteration of the nearest kernel (2: each LDS centroid fragment feeds two MFMA chains;
# 3 / 4 at D = 128 only, see _rg; D = 256 always runs 1)
# default 3 (D = 128; D = 64 runs 2): tools/kmeans_nearest_bench.py RG_AB, 1e8 rows x 201 candidates, counts mode
# 7.03-7.20 ms (RG 2) -> 6.86-6.88 (RG 3), identical results (profiles/kmeans_init_r6.txt)
NEAREST_RG = int(os.environ.get("ALINK_KMEANS_NEAREST_RG", "3"))
NEAREST_GRID = int(os.environ.get("ALINK_KMEANS_NEAREST_GRID", "2"))     # persistent workgroups per CU


def _rg(d: int, m: int) -> int:
    """32-row groups per wave iteration of the nearest kernel: NEAREST_RG (1..4; 3 and 4 only at D = 128, without
    the fragment prefetch) when more than one centroid block is scanned, else 1."""
    if m <= 32 or d > 128 or NEAREST_RG <= 1:
        return 1
    return NEAREST_RG if d == 128 else 2


def nearest_supported(X: torch.Tensor) -> bool:
    return (X.is_cuda and X.dtype == torch.bfloat16 and X.dim() == 2 and X.shape[1] in NEAREST_DIMS
            and X.shape[0] > 0 and X.is_contiguous() and X.data_ptr() % 16 == 0)


def par_pick_hip(cost: torch.Tensor, first_row: int, key: int, thre: float) -> torch.Tensor:
    """k-means|| oversampling draw in one launch (``csrc/kmeans_nearest.hip`` ``kmeans_par_pick_kernel``): the
    sorted local indices i with ``u(first_row + i) < cost[i] * thre`` — the same picks, bit for bit, as the torch
    expression over ``models/clustering/kmeans._row_uniform`` (splitmix64 of the global row index, ``key`` being
    its signed 64-bit round key), without materialising the [N] uniforms.  One 8-byte read for the pick count."""
    L = _lib.require()
    dev = cost.device
    n = int(cost.shape[0])
    cost = cost.contiguous()
    cap = 4096
    while True:
        out = torch.empty(cap, dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        rc = L.alink_kmeans_par_pick(cost.data_ptr(), n, int(first_row), int(key), float(thre), out.data_ptr(),
                                     cap, cnt.data_ptr(), _lib.stream_ptr(dev))
        if rc != 0:
            raise RuntimeError(f"alink_kmeans_par_pick failed: {rc}")
        c = int(cnt.item())
        if c <= cap:
            return torch.sort(out[:c]).values
        cap = c


def seed_ref_hip(D: torch.Tensor, w: torch.Tensor, U: torch.Tensor, k: int, idx0: int = -1,
                 r0: float = 0.0, prof: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """The reference seeding rule's k picks over n <= 4096 k-means|| candidates in one launch
    (``csrc/kmeans_nearest.hip`` ``kmeans_seed_ref_kernel``): D [n, n] fp64 plain distances, w [n] weights,
    U [k-1] the picks' uniforms.  ``idx0 < 0``: the first pick too, from the uniform ``r0`` over the sequential
    cumulative weights.  Returns (chosen int64 [k], mintot fp64 [1]) on the device, nothing read back."""
    L = _lib.require()
    n = int(D.shape[0])
    chosen = torch.empty(k, dtype=torch.int64, device=D.device)
    mintot = torch.full((1,), float("inf"), dtype=torch.float64, device=D.device)
    Dc, wc, Uc = D.contiguous(), w.contiguous(), U.contiguous()
    rc = L.alink_kmeans_seed_ref2(Dc.data_ptr(), wc.data_ptr(), Uc.data_ptr(), n, int(k), int(idx0), float(r0),
                                  chosen.data_ptr(), mintot.data_ptr(), None if prof is None else prof.data_ptr(),
                                  _lib.stream_ptr(D.device))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_seed_ref2 failed: {rc}")
    return chosen, mintot


LOCAL_LLOYD_NMAX = 4096


def local_lloyd_lds(n: int, d: int, k: int) -> int:
    """LDS bytes of ``kmeans_local_lloyd_kernel`` (csrc/kmeans_nearest.hip local_lloyd_lds)."""
    return (k * (d + 1) + 2 * k + 2 * n) * 8 + (2 * n + k + 1) * 4


def local_lloyd_ok(samples: torch.Tensor, k: int) -> bool:
    """The one-workgroup weighted Lloyd applies: fp64 [n, d] candidates on the GPU, n <= 4096, and the
    centroids (rows padded to d + 1) plus the per-sample state fit the 160 KiB LDS."""
    if not (samples.is_cuda and samples.dtype == torch.float64 and samples.dim() == 2):
        return False
    n, d = samples.shape
    return (1 <= n <= LOCAL_LLOYD_NMAX and d >= 1 and 1 <= k <= n and local_lloyd_lds(n, d, k) <= 160 * 1024
            and _lib.available())


def local_lloyd_hip(X: torch.Tensor, w: torch.Tensor, k: int, C: Optional[torch.Tensor] = None,
                    chosen: Optional[torch.Tensor] = None, assign: Optional[torch.Tensor] = None,
                    max_iter: int = 30, mintot: Optional[torch.Tensor] = None, prof: Optional[torch.Tensor] = None):
    """Weighted Lloyd (EUCLIDEAN) on the k-means|| candidates in ONE workgroup, every iteration on the chip
    (``csrc/kmeans_nearest.hip`` ``kmeans_local_lloyd_kernel``): runs until the assignment is unchanged, a cluster
    is empty (the caller refills it and calls again with ``C`` / ``assign``) or ``max_iter`` iterations.  The
    start centroids are ``C`` (updated in place) or the rows ``X[chosen]``.  Returns (C [k, d], assign int64 [n],
    status fp64 [6] = iterations, changed, empty, non-finite input, mintot, chosen[0], live uint8 [k]), all on the
    device: the caller reads ``status`` once.  ``prof``: int64 [50] receives 100 MHz wall-clock stamps (setup, then
    six phases per iteration for the first 8; tools/kmeans_local_bench.py)."""
    L = _lib.require()
    n, d = X.shape
    dev = X.device
    Xc = X.contiguous()
    wc = w.to(torch.float64).contiguous()
    if C is None:
        if chosen is None:
            raise ValueError("local_lloyd_hip needs C or chosen")
        C = torch.empty((k, d), dtype=torch.float64, device=dev)
    if assign is None:
        assign = torch.full((n,), -1, dtype=torch.int64, device=dev)
    ct = (k + 63) // 64
    bd = torch.empty(n * ct, dtype=torch.float64, device=dev)
    bi = torch.empty(n * ct, dtype=torch.int32, device=dev)
    status = torch.zeros(6, dtype=torch.float64, device=dev)
    live = torch.empty(k, dtype=torch.uint8, device=dev)
    ch = chosen.contiguous() if chosen is not None else None
    rc = L.alink_kmeans_local_lloyd(Xc.data_ptr(), wc.data_ptr(), n, d, int(k), None if ch is None else ch.data_ptr(),
                                    C.data_ptr(), assign.data_ptr(), bd.data_ptr(), bi.data_ptr(), int(max_iter),
                                    None if mintot is None else mintot.data_ptr(), status.data_ptr(), live.data_ptr(),
                                    None if prof is None else prof.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_kmeans_local_lloyd failed: {rc}")
    return C, assign, status, live


def nearest_hip(X: torch.Tensor, C: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(index int32 [N], squared Euclidean distance float32 [N]) of every row's nearest centroid —
    ``csrc/kmeans_nearest.hip``: one MFMA pass over X per 256 centroids (k-means|| seeding, predict).
    Centroids are rounded to bf16 (k-means|| candidates are rows of X, so exactly representable)."""
    L = _lib.require()
    if not nearest_supported(X):
        raise ValueError("nearest_hip needs contiguous bf16 [N, D] on GPU with D in (64, 128, 256)")
    n, d = X.shape
    Cb = C.to(device=X.device, dtype=torch.bfloat16).contiguous()
    if Cb.shape[1] != d or Cb.shape[0] == 0:
        raise ValueError("centroid shape mismatch")
    chalf = (0.5 * (Cb.float() ** 2).sum(1)).contiguous()
    idx = torch.empty(n, dtype=torch.int32, device=X.device)
    d2 = torch.empty(n, dtype=torch.float32, device=X.device)
    grid = NEAREST_GRID * _num_cus(X.device)
    st = _lib.stream_ptr(X.device)
    for c0 in range(0, Cb.shape[0], NEAREST_CHUNK):
        m = min(NEAREST_CHUNK, Cb.shape[0] - c0)
        # one centroid block (the first k-means|| cost pass): load-bound, RG = 1 measured 2 % ahead
        rg = _rg(d, m)
        rc = L.alink_kmeans_nearest_bf16_rg(X.data_ptr(), n, d, Cb[c0].data_ptr(), chalf[c0].data_ptr(), m, c0,
                                            idx.data_ptr(), d2.data_ptr(), int(c0 > 0), grid, rg, None, st)
        if rc != 0:
            raise RuntimeError(f"alink_kmeans_nearest_bf16 failed: {rc}")
    return idx, d2
