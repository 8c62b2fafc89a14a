"""Loader for the in-tree HIP kernel library (``libalink_hip.so``, built for gfx950 by ``build_native.py``).

The library exposes a plain C ABI (raw device pointers + the caller's HIP stream), called through
``ctypes``: no torch C++ ABI coupling, and every launch goes on torch's current stream so kernels
compose with RCCL collectives and hipGraph capture.

On a GPU box a missing/unloadable library is an error (``require()`` raises) — ops never silently fall
back to PyTorch when a GPU is present, unless ``ALINK_ALLOW_TORCH_FALLBACK=1`` is set explicitly.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  (loads torch's HIP runtime first; our .so resolves libamdhip64.so.7 to it)

__all__ = ["lib", "require", "available", "LIB_PATH", "stream_ptr"]

LIB_PATH = os.environ.get("ALINK_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libalink_hip.so")
_lib: Optional[ctypes.CDLL] = None
_err: Optional[str] = None


def _load():
    global _lib, _err
    if _lib is not None or _err is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        _err = f"{LIB_PATH} not built (run python build_native.py)"
        return None
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on box
        _err = f"cannot load {LIB_PATH}: {e}"
        return None
    c_i64, c_int, c_vp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
    L.alink_kmeans_reduce_slabs.argtypes = [c_vp, c_vp, c_int, c_int, c_vp, c_vp]
    L.alink_kmeans_reduce_slabs.restype = c_int
    L.alink_kmeans_prep_centroids.argtypes = [c_vp, c_int, c_vp, c_vp, c_vp]
    L.alink_kmeans_prep_centroids.restype = c_int
    for name, argtypes in _EXTRA_SIGNATURES.items():
        if hasattr(L, name):
            getattr(L, name).argtypes = argtypes
            getattr(L, name).restype = c_int
    # every entry point is a ``kernel`` span on the timeline when utils.trace is on (host launch cost + device
    # time from HIP events on the caller's stream); one flag check per call otherwise
    from ..utils import trace
    for name in ["alink_kmeans_reduce_slabs", "alink_kmeans_prep_centroids"] + list(_EXTRA_SIGNATURES):
        if hasattr(L, name) and not name.endswith(("_grid", "_pad", "_padded_rank", "_kmax", "_alloc", "_free")):
            setattr(L, name, trace.traced_call(getattr(L, name), name[len("alink_"):]))
    _lib = L
    return _lib


_c_i64, _c_int, _c_vp, _c_f = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_float
_c_d = ctypes.c_double
# signatures of further kernels (registered when present in the library)
_EXTRA_SIGNATURES = {
    "alink_tree_gather_rows": [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp],
    "alink_tree_hist_fm": [_c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_int,
                           _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_int],
    "alink_tree_hist_f32": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_int, _c_int,
                            _c_vp],
    "alink_tree_node_sums": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_int, _c_vp],
    "alink_tree_route": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp],
    "alink_kmeans_assign_accum_bf16_v7": [_c_vp, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                          _c_int],
    "alink_kmeans_v7_grid": [_c_i64, _c_int],
    "alink_kmeans_assign_accum_bf16_v10": [_c_vp, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                           _c_int],
    "alink_kmeans_assign_accum_bf16_v10s": [_c_vp, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                            _c_int, _c_vp],
    "alink_kmeans_assign_accum_bf16_v10d": [_c_vp, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                            _c_int, _c_vp, _c_int, _c_d],
    "alink_kmeans_v10_grid": [_c_i64, _c_int],
    "alink_kmeans_reduce_slabs2": [_c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp],
    "alink_tree_predict": [_c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_int,
                           _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_tree_codes": [_c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp],
    "alink_gbdt_rank_stats": [_c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_kmeans_seed_ref": [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp],
    "alink_kmeans_seed_ref2": [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_d, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_kmeans_local_lloyd": [_c_vp, _c_vp, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp,
                                 _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_kmeans_par_pick": [_c_vp, _c_i64, _c_i64, _c_i64, _c_d, _c_vp, _c_i64, _c_vp, _c_vp],
    "alink_kmeans_nearest_bf16": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_int,
                                  _c_int, _c_vp],
    "alink_kmeans_cost1_bf16": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_vp],
    "alink_kmeans_cost1_bf16_sum": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp],
    "alink_kmeans_nearest_bf16_rg": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_int,
                                     _c_int, _c_int, _c_vp, _c_vp],
    "alink_linear_grad_f64": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_d, _c_vp, _c_int, _c_vp,
                              _c_vp],
    "alink_linear_grad_pad": [_c_int],
    "alink_linear_search_f64": [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_d, _c_d, _c_int, _c_vp,
                                _c_int, _c_vp, _c_vp],
    "alink_kmeans_update": [_c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp],
    "alink_kmeans_update2": [_c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_d, _c_vp,
                             ctypes.c_uint64, _c_vp],
    "alink_kmeans_host_stat_alloc": [ctypes.POINTER(_c_vp), ctypes.POINTER(_c_vp)],
    "alink_kmeans_host_stat_free": [_c_vp],
    "alink_kmeans_accum_bf16": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_kmeans_accum_f32": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_kmeans_accum_kmax": [_c_int],
    "alink_kmeans_accum_mfma_bf16": [_c_vp, _c_i64, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_linear_grad_wide_f64": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_d, _c_vp, _c_int, _c_vp,
                                   _c_vp],
    "alink_csr_row_deriv_f64": [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_d, _c_vp, _c_vp, _c_vp],
    "alink_csc_gather_f64": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp],
    "alink_ftrl_check_indices": [_c_vp, _c_i64, _c_i64, _c_vp, _c_int, _c_vp],
    "alink_ftrl_hogwild_f64": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_d, _c_d, _c_d, _c_d, _c_int,
                               _c_vp],
    "alink_ftrl_partial_margin_f64": [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_vp, _c_int, _c_vp],
    "alink_ftrl_coord_update_f64": [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_d, _c_d,
                                    _c_d, _c_d, _c_i64, _c_int, _c_vp],
    "alink_ftrl_coord_scan_f64": [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_d, _c_d,
                                  _c_d, _c_d, _c_int, _c_vp],
    "alink_ftrl_coord_long_f64": [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_d, _c_d,
                                  _c_d, _c_d, _c_int, _c_vp],
    "alink_ftrl_prox_f64": [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_d, _c_d, _c_d, _c_d, _c_int, _c_vp],
    "alink_murmur3_utf8_index": [_c_vp, _c_vp, _c_i64, _c_vp, _c_int, ctypes.c_uint32, _c_i64, _c_vp, _c_vp, _c_vp],
    "alink_murmur3_multi_index": [_c_vp, _c_int, _c_i64, ctypes.c_uint32, _c_i64, _c_vp, _c_vp, _c_vp],
    "alink_murmur3_bytes": [_c_vp, _c_vp, _c_i64, ctypes.c_uint32, _c_vp, _c_vp],
    "alink_vector_assemble": [_c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp],
    "alink_murmur3_index": [_c_vp, _c_vp, _c_i64, _c_vp, _c_int, ctypes.c_uint32, _c_i64, _c_vp, _c_vp, _c_vp],
    "alink_csr_assemble": [_c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_csr_mv_f64": [_c_vp, _c_vp, _c_int, _c_vp, _c_i64, _c_vp, _c_vp, _c_d, _c_vp],
    "alink_tree_quantize": [_c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_int, _c_vp,
                            _c_vp],
    "alink_tree_quantize_f32": [_c_vp, _c_vp, _c_vp, _c_int, _c_i64, _c_int, _c_vp, _c_int, _c_int, _c_vp, _c_vp],
    "alink_tree_split": [_c_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_vp, _c_d, _c_d, _c_d, _c_d, _c_vp,
                         _c_vp, _c_vp],
    "alink_gbdt_split": [_c_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_d, _c_d, _c_vp, _c_vp,
                         _c_vp],
    "alink_als_fused_solve": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_f, _c_vp, _c_vp, _c_vp, _c_vp,
                              _c_vp, _c_vp],
    "alink_als_mfma_solve": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_f, _c_vp, _c_vp, _c_vp, _c_vp,
                              _c_vp, _c_vp],
    "alink_als_heavy_solve": [_c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_f, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp,
                              _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp],
    "alink_als_woodbury16_mfma": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_als_woodbury_solve": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                 _c_vp],
    "alink_als_padded_rank": [_c_int],
    "alink_topk_cross_f32": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_int, _c_i64,
                             _c_vp],
    "alink_colstats": [_c_vp, _c_i64, _c_int, _c_int, _c_int, _c_vp, _c_vp],
    "alink_fm_forward_f64": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_d, _c_vp, _c_vp, _c_vp],
    "alink_fm_coord_update_f64": [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                  _c_vp, _c_vp, _c_vp, _c_d, _c_d, _c_d, _c_d, _c_vp],
    "alink_w2v_sg_hs_f32": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                            _c_int, _c_f, _c_int, _c_vp],
    "alink_lda_gibbs": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_d, _c_d, _c_d, _c_vp, _c_vp,
                        _c_int, _c_vp],
    "alink_lda_estep": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_int, _c_d, _c_vp, _c_vp, _c_vp,
                        _c_vp],
    "alink_gbdt_grad_stats": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp],
    "alink_gbdt_leaf_update": [_c_vp, _c_vp, _c_vp, _c_int, _c_i64, _c_vp],
    "alink_col_transform": [_c_vp, _c_i64, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_d, _c_d, _c_vp, _c_vp],
    "alink_softmax_grid": [_c_i64],
    "alink_softmax_grad_f64": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp],
    "alink_softmax_search_f64": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_d, _c_int, _c_vp, _c_vp],
    "alink_gmm_grid": [_c_i64],
    "alink_gmm_estep_f64": [_c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp],
    "alink_softmax_full_grad_f64": [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp],
    "alink_bias_sigmoid_f64": [_c_vp, _c_i64, _c_int, _c_vp, _c_vp],
    "alink_sigmoid_bwd_f64": [_c_vp, _c_vp, _c_i64, _c_vp],
    "alink_als_gram_f32": [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_int, _c_f, _c_vp, _c_vp, _c_vp],
}


def lib() -> Optional[ctypes.CDLL]:
    return _load()


def available() -> bool:
    return _load() is not None


def require() -> ctypes.CDLL:
    L = _load()
    if L is None:
        raise RuntimeError(f"alink_amd HIP kernels unavailable: {_err}")
    return L


def torch_fallback_allowed() -> bool:
    return os.environ.get("ALINK_ALLOW_TORCH_FALLBACK", "0") == "1"


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
