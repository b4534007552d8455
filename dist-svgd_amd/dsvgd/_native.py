"""ctypes binding of libdsvgd_hip.so (the C ABI declared in include/dsvgd.h).

There is deliberately no fallback: if the HIP library is missing or cannot be
loaded, every compute entry point raises :class:`NativeUnavailable`.  The
SVGD math runs only in the gfx950 kernels.
"""
import ctypes
import os

import torch

ABI_VERSION = 4
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libdsvgd_hip.so")

_c = ctypes
_p = _c.c_void_p
_i64 = _c.c_int64
_f = _c.c_float
_f64 = _c.c_double
_int = _c.c_int



class GramPart(ctypes.Structure):
    """Mirror of dsvgd_gram_part (include/dsvgd.h)."""
    _fields_ = [("row_off", _i64), ("rows", _i64), ("col0", _i64), ("cols", _i64),
                ("kind", ctypes.c_int32), ("weight2", ctypes.c_int32)]


class PhiPart(ctypes.Structure):
    """Mirror of dsvgd_phi_part (include/dsvgd.h)."""
    _fields_ = [("ky", _p), ("rs", _p), ("ldk", _i64), ("row_off", _i64), ("rows", _i64),
                ("splits", _i64)]


# name -> (restype, argtypes); must mirror include/dsvgd.h exactly
SIGNATURES = {
    "dsvgd_abi_version": (_int, []),
    "dsvgd_last_error": (_c.c_char_p, []),
    "dsvgd_select_state_bytes": (_c.c_size_t, []),
    "dsvgd_pad128": (_i64, [_i64]),
    "dsvgd_dp": (_i64, [_i64]),
    "dsvgd_ldy": (_i64, [_i64]),
    "dsvgd_colmean_workspace_floats": (_c.c_size_t, [_i64, _i64]),
    "dsvgd_colmean": (_int, [_p, _i64, _i64, _i64, _p, _p, _p]),
    "dsvgd_colcenter": (_int, [_p, _i64, _i64, _i64, _p, _p]),
    "dsvgd_pack": (_int, [_p, _i64, _p, _i64, _f, _p, _i64, _i64, _i64, _p, _i64, _p, _p]),
    "dsvgd_pack_blocks": (_i64, [_i64]),
    "dsvgd_pack_max_ldy": (_i64, []),
    "dsvgd_pack_h2": (_int, [_p, _i64, _p, _i64, _f, _p, _i64, _i64, _i64, _p, _i64, _p, _p, _p,
                             _p, _p]),
    "dsvgd_sqdist": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _int, _p, _p, _p]),
    "dsvgd_sqdist_direct": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _int, _p, _p,
                                   _p]),
    "dsvgd_select_init": (_int, [_p, _i64, _i64, _p]),
    "dsvgd_radix_hist": (_int, [_p, _i64, _p, _int, _p, _i64, _p]),
    "dsvgd_radix_pick": (_int, [_p, _int, _p]),
    "dsvgd_sample_sqdist": (_int, [_p, _i64, _i64, _i64, _i64, _c.c_uint64, _p, _p]),
    "dsvgd_bracket_init": (_int, [_p, _i64, _p, _p, _i64, _p]),
    "dsvgd_sample_bracket": (_int, [_p, _i64, _i64, _i64, _i64, _c.c_uint64, _i64, _i64, _p, _p,
                                    _p, _p, _i64, _i64, _p]),
    "dsvgd_sample_sqdist_range": (_int, [_p, _i64, _i64, _i64, _i64, _c.c_uint64, _i64, _i64, _p,
                                         _p]),
    "dsvgd_sample_bracket_select": (_int, [_p, _i64, _i64, _i64, _p, _p, _p, _i64, _i64, _p]),
    "dsvgd_bracket_totals": (_int, [_p, _p, _p]),
    "dsvgd_bracket_check": (_int, [_p, _p]),
    "dsvgd_set_bandwidth": (_int, [_p, _f, _p]),
    "dsvgd_phi_splits": (_i64, [_i64, _i64, _i64]),
    "dsvgd_phi_set_symrow": (_int, [_int]),
    "dsvgd_phi_set_finish_vec": (_int, [_int]),
    "dsvgd_gram_set_rs": (_int, [_int]),
    "dsvgd_gram_set_group": (_int, [_int]),
    "dsvgd_set_cu_reserve": (_int, [_int]),
    "dsvgd_gram_debug_stamps": (_int, [_p]),
    "dsvgd_phi_splits_sym": (_i64, [_i64, _i64]),
    "dsvgd_phi_set_xmap": (_int, [_int]),
    "dsvgd_gsw_set_inc": (_int, [_int]),
    "dsvgd_phi_set_gxd_w1": (_int, [_int]),
    "dsvgd_logreg_set_fused": (_int, [_int]),
    "dsvgd_phi_mm": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _p]),
    "dsvgd_phi_mm_gated": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _p,
                                  _p]),
    "dsvgd_ysplit_bytes": (_i64, [_i64, _i64]),
    "dsvgd_ysplit": (_int, [_p, _i64, _i64, _p, _int, _p, _p]),
    "dsvgd_rowsplit_bytes": (_i64, [_i64, _i64]),
    "dsvgd_rowsplit": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _p, _int, _p]),
    "dsvgd_sqdist_x3": (_int, [_p, _p, _i64, _i64, _i64, _i64, _p, _i64, _int, _p, _p, _int, _p]),
    "dsvgd_phi_mm_x3": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _int,
                                _int, _p, _p]),
    "dsvgd_h2_colscale_workspace_floats": (_c.c_size_t, [_i64, _i64]),
    "dsvgd_h2_colscale": (_int, [_p, _i64, _i64, _i64, _p, _p, _p]),
    "dsvgd_h2_colscale_guarded": (_int, [_p, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "dsvgd_h2_scales": (_int, [_p, _p, _i64, _i64, _i64, _i64, _p, _p]),
    "dsvgd_h2_image_bytes": (_i64, [_i64, _i64]),
    "dsvgd_h2_ysplit": (_int, [_p, _i64, _i64, _p, _p, _p]),
    "dsvgd_h2_rowsplit": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "dsvgd_h2_rowsplit_rows": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "dsvgd_h2_rowscale": (_int, [_p, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "dsvgd_h2_rowimage": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _p, _p, _p, _p]),
    "dsvgd_sqdist_h2": (_int, [_p, _p, _i64, _i64, _i64, _i64, _p, _i64, _int, _p, _p, _int, _p,
                               _p]),
    "dsvgd_phi_mm_h2": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _i64, _p, _i64, _p, _int,
                               _p, _p, _p]),
    "dsvgd_phi_finish": (_int, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p, _f,
                                _f, _p, _i64, _p, _i64, _p, _i64, _p]),
    "dsvgd_phi_direct": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p, _f, _f, _p,
                                _i64, _p, _i64, _p, _i64, _p, _i64, _p]),
    "dsvgd_phi_row": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _f, _p, _p, _p]),
    "dsvgd_phi_row_blocks": (_i64, [_i64, _i64]),
    "dsvgd_phi_row_split": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _f, _p, _p, _p, _i64,
                                   _p]),
    "dsvgd_gs_block_rows": (_i64, []),
    "dsvgd_gs_splits": (_i64, [_i64]),
    "dsvgd_gs_block_part": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p, _p, _i64, _p]),
    "dsvgd_gs_block_sweep": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p, _f, _p, _i64,
                                    _p, _i64, _p, _i64, _int, _p, _p, _f, _p]),
    "dsvgd_w2_cost": (_int, [_p, _i64, _i64, _p, _i64, _i64, _i64, _p, _i64, _p]),
    "dsvgd_w2_workspace_bytes": (_c.c_size_t, [_i64, _i64]),
    "dsvgd_w2_cost_h2_workspace_bytes": (_c.c_size_t, [_i64, _i64, _i64]),
    "dsvgd_w2_cost_h2": (_int, [_p, _i64, _i64, _p, _i64, _i64, _i64, _p, _i64, _p, _c.c_float, _p,
                                 _p]),
    "dsvgd_w2_assign": (_int, [_p, _i64, _i64, _i64, _p, _i64, _int, _p, _p, _p]),
    "dsvgd_w2_assign_warm": (_int, [_p, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _p]),
    "dsvgd_w2_set_cost_nt": (_int, [_int]),
    "dsvgd_w2_set_cost_lines": (_int, [_int]),
    "dsvgd_w2_assign_stat": (_int, [_p, _i64, _i64, _i64, _p, _i64, _int, _p, _p, _p, _p, _p]),
    "dsvgd_w2_trace": (_i64, [_p, _i64]),
    "dsvgd_w2_set_keep": (_int, [_int]),
    "dsvgd_w2_set_theta": (_f64, [_f64]),
    "dsvgd_w2_tail_stats": (_i64, [_p]),
    "dsvgd_w2_set_tail_debug": (_int, [_int]),
    "dsvgd_w2_set_fuse_first": (_int, [_int]),
    "dsvgd_w2_grad": (_int, [_p, _i64, _i64, _p, _i64, _i64, _i64, _p, _f, _p, _i64, _p]),
    "dsvgd_score_gaussian": (_int, [_p, _i64, _i64, _i64, _p, _p, _f, _p, _i64, _p]),
    "dsvgd_score_gmm": (_int, [_p, _i64, _i64, _i64, _f, _p, _i64, _p]),
    "dsvgd_logreg_workspace_bytes": (_c.c_size_t, [_i64, _i64, _i64]),
    "dsvgd_score_logreg": (_int, [_p, _i64, _i64, _i64, _p, _i64, _p, _i64, _f, _p, _i64, _p,
                                  _p]),
    "dsvgd_score_logreg_engine": (_int, [_p, _i64, _i64, _i64, _p, _i64, _p, _i64, _f, _p, _i64,
                                         _p, _int, _p]),
    "dsvgd_logreg_prepare": (_int, [_p, _i64, _p, _i64, _i64, _i64, _p, _int, _p]),
    "dsvgd_score_logreg_prepared": (_int, [_p, _i64, _i64, _i64, _i64, _f, _p, _i64, _p, _int,
                                           _p]),
    "dsvgd_score_logreg_prior": (_int, [_p, _i64, _i64, _i64, _i64, _f, _f, _p, _i64, _p, _int,
                                        _p]),
    "dsvgd_logreg_predict_workspace_bytes": (_c.c_size_t, [_i64, _i64, _i64]),
    "dsvgd_logreg_predict": (_int, [_p, _i64, _i64, _i64, _p, _i64, _i64, _p, _p, _p]),
    # the wide blocked Gauss-Seidel sweep (ABI 4)
    "dsvgd_gsw_block_rows": (_i64, [_i64, _int]),
    "dsvgd_gsw_debug": (_int, [_int]),
    "dsvgd_h2_rowsplit_rows_range": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _p, _p, _i64, _i64,
                                            _p]),
    "dsvgd_gs_mask": (_int, [_p, _i64, _i64, _i64, _p]),
    "dsvgd_gs_mask_cols": (_int, [_p, _i64, _i64, _i64, _i64, _p]),
    "dsvgd_debug_spin": (_int, [_i64, _p]),
    "dsvgd_gsw_group_corr": (_int, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _i64,
                                    _p, _p, _i64, _p, _p]),
    "dsvgd_gsw_block_sweep": (_int, [_p, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _i64,
                                     _p, _f, _p, _i64, _p, _p, _i64, _p, _i64, _int, _p, _p, _f,
                                     _p, _i64, _p, _i64, _p]),
    # the pair-split layout (ABI 4)
    "dsvgd_sqdist_h2_parts": (_int, [_p, _p, _i64, _i64, _i64, _i64, _p, _i64, _int, _p, _p, _p,
                                     _int, _p, _p, _p]),
    "dsvgd_radix_hist_wmap": (_int, [_p, _i64, _i64, _p, _int, _p, _p, _p]),
    "dsvgd_phi_h2_window": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _i64, _p,
                                   _i64, _p, _p, _p, _int, _p]),
    "dsvgd_phi_h2_transposed": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _i64,
                                       _p, _i64, _p, _p, _p, _int, _p]),
    "dsvgd_phi_h2_transposed_blocks": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _i64,
                                              _i64, _p, _p, _i64, _i64, _p, _p, _int, _p]),
    "dsvgd_phi_h2_transposed_blocks_split": (_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _i64,
                                                    _i64, _i64, _i64, _p, _p, _i64, _i64, _p, _p,
                                                    _int, _p]),
    "dsvgd_phi_partial_reduce_blocks": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _i64,
                                               _i64, _p]),
    "dsvgd_phi_partial_reduce": (_int, [_p, _i64, _p, _i64, _i64, _i64, _p, _i64, _p, _p]),
    "dsvgd_phi_finish_parts": (_int, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p, _f,
                                      _f, _p, _i64, _p, _i64, _p, _i64, _p, _int, _p, _i64, _p]),
}


class NativeUnavailable(RuntimeError):
    """libdsvgd_hip.so is missing or unusable (no silent fallback exists)."""


class NativeError(RuntimeError):
    """A libdsvgd_hip.so entry point returned an error code."""


_lib = None


def load():
    """Load (once) and return the ctypes library with typed entry points."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(
            "libdsvgd_hip.so not found at %s -- build it with `make -C dist-svgd_amd` "
            "(or __graft_entry__.build()); dsvgd has no non-HIP compute path" % LIB_PATH)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - environment specific
        raise NativeUnavailable("cannot load %s: %s" % (LIB_PATH, e))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dsvgd_abi_version() != ABI_VERSION:
        raise NativeUnavailable("ABI version mismatch")
    _lib = lib
    return lib


def call(name, *args):
    """Invoke entry point `name`; raise NativeError on a nonzero return code."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise NativeError("%s failed (%d): %s" % (name, rc, lib.dsvgd_last_error().decode()))


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("dsvgd kernels need device (HIP) tensors, got %s" % t.device)
    return t.data_ptr()


def ld(t):
    """Leading dimension (row stride, elements) of a row-major 2-D tensor; a
    (n, 1) tensor is row-major whatever its column stride says."""
    if t.dim() != 2:
        raise ValueError("expected a 2-D tensor, got shape %s" % (tuple(t.shape),))
    if t.shape[1] != 1 and t.stride(1) != 1:
        raise ValueError("tensor must be row-major (stride(1) == 1), got strides %s"
                         % (t.stride(),))
    if t.dtype != torch.float32:
        raise ValueError("dsvgd kernels take float32 tensors, got %s" % t.dtype)
    return max(t.stride(0), t.shape[1]) if t.shape[0] == 1 else t.stride(0)


def stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(device):
    dev = torch.device(device)
    if dev.type != "cuda":
        raise NativeUnavailable("dsvgd runs on MI355X (HIP) devices only; got device %s" % dev)
    if not torch.cuda.is_available():
        raise NativeUnavailable("no HIP device visible; dsvgd has no CPU compute path")
    load()
    return dev
