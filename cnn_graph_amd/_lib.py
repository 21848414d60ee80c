"""ctypes binding of libcheb_mi355.so (the C ABI declared in include/cheb_mi355.h).

The HIP library is the only compute path: if it is missing this module raises
ImportError -- there is no CPU or PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# CG_LIB_PATH: load an alternative in-tree build (kernel-variant experiments)
LIB_PATH = os.environ.get("CG_LIB_PATH") or os.path.join(_HERE, "libcheb_mi355.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "cheb_mi355.h")

CG_OK, CG_ERR_ARG, CG_ERR_HIP, CG_ERR_UNSUPPORTED, CG_ERR_ALLOC, CG_ERR_COMM = range(6)
CG_PATH_AUTO, CG_PATH_RESIDENT, CG_PATH_STREAM = 0, 1, 2
CG_ACT_NONE, CG_ACT_RELU, CG_ACT_TANH = 0, 1, 2
PATHS = {"auto": CG_PATH_AUTO, "resident": CG_PATH_RESIDENT, "stream": CG_PATH_STREAM}
CG_VARIANT_AUTO, CG_VARIANT_CLASSIC, CG_VARIANT_UNFUSED_DW, CG_VARIANT_NARROW = 0, 1, 2, 3
CG_VARIANT_STEPS = 4
VARIANTS = {"auto": CG_VARIANT_AUTO, "classic": CG_VARIANT_CLASSIC,
            "unfused_dw": CG_VARIANT_UNFUSED_DW, "narrow": CG_VARIANT_NARROW,
            "steps": CG_VARIANT_STEPS}
CG_BASIS_ROWS, CG_BASIS_ORDERS, CG_BASIS_PLANES = 0, 1, 2
BASIS_LAYOUTS = {"rows": CG_BASIS_ROWS, "orders": CG_BASIS_ORDERS, "planes": CG_BASIS_PLANES}
# kernel-selection options (cg_set_option; include/cheb_mi355.h CG_OPT_*)
OPTIONS = {"dw_direct": 0, "dw_w2": 1, "dw_waves": 2, "spmm_pw": 3, "grp16": 4, "grp_pc": 5,
           "clen_dy": 6, "seq_xpre": 7, "dw_x3": 8, "gemm_x3": 9}


class CGError(RuntimeError):
    """A non-zero status from libcheb_mi355 (message from cg_last_error())."""

    def __init__(self, func, code, msg):
        super().__init__(f"{func} failed with status {code}: {msg}")
        self.code = code


_c_int, _c_i32, _c_i64, _c_sz = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
_vp, _fp = ctypes.c_void_p, ctypes.c_void_p  # device pointers are passed as void*
_ip32 = ctypes.POINTER(ctypes.c_int32)
_fp32 = ctypes.POINTER(ctypes.c_float)

_SIGNATURES = {
    "cg_version": ([], _c_int),
    "cg_last_error": ([], ctypes.c_char_p),
    "cg_plan_create": ([ctypes.POINTER(_vp), _c_int, _c_i32, _c_i64, _ip32, _ip32, _fp32,
                        _ip32, _ip32, _fp32], _c_int),
    "cg_plan_destroy": ([_vp], _c_int),
    "cg_plan_set_path": ([_vp, _c_int], _c_int),
    "cg_plan_set_variant": ([_vp, _c_int], _c_int),
    "cg_plan_query_path": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_int)], _c_int),
    "cg_cheb_workspace_bytes": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_sz),
                                 ctypes.POINTER(_c_sz)], _c_int),
    "cg_cheb_forward": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp],
                        _c_int),
    "cg_cheb_backward": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _c_sz,
                          _vp], _c_int),
    "cg_cheb_forward_ex": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _c_i32, _vp, _vp, _vp,
                            _c_sz, _vp], _c_int),
    "cg_cheb_backward_ex": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp,
                             _c_i32, _vp, _vp, _vp, _c_sz, _vp], _c_int),
    "cg_cheb_basis_elems": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_i64)],
                            _c_int),
    "cg_cheb_forward_layout": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _c_i32, _c_i32,
                                _vp, _vp, _vp, _c_sz, _vp], _c_int),
    "cg_cheb_backward_layout": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _c_i32, _c_i32, _vp,
                                 _vp, _vp, _c_i32, _vp, _vp, _vp, _c_sz, _vp], _c_int),
    "cg_cheb_forward_adam": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp,
                              ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                              _c_i32, ctypes.c_float, _vp, _vp, _vp, _c_i32, _vp, _vp, _vp, _c_sz,
                              _vp], _c_int),
    "cg_cheb_backward_adam_layout": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp,
                                      _vp, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, _c_i32, ctypes.c_float, _vp,
                                      _c_sz, _vp], _c_int),
    "cg_mse_loss_workspace_bytes": ([_c_i64, ctypes.POINTER(_c_sz)], _c_int),
    "cg_mse_loss": ([_vp, _vp, _c_i64, _vp, _vp, _vp, _c_sz, _vp], _c_int),
    "cg_mse_loss_ema": ([_vp, _vp, _c_i64, _vp, _vp, _vp, ctypes.c_float, _vp, _c_sz, _vp], _c_int),
    "cg_slice_channels": ([_vp, _c_i64, _c_i32, _c_i32, _c_i32, _vp, _vp], _c_int),
    "cg_stack_merge_forward": ([_c_i32, _c_i32, _c_i32, _vp, _vp, _c_i32, _vp, _vp], _c_int),
    "cg_stack_merge_backward": ([_c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp], _c_int),
    "cg_weight_grad_workspace_bytes": ([_c_i64, _c_i32, _c_i32, ctypes.POINTER(_c_sz)], _c_int),
    "cg_weight_grad": ([_c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _c_i32, _vp, _c_sz, _vp], _c_int),
    "cg_weight_grad_planes": ([_c_i64, _c_i32, _c_i32, _c_i32, _vp, _c_i64, _vp, _vp, _c_i32, _vp, _c_sz,
                               _vp], _c_int),
    "cg_lstm_weight_grads_workspace_bytes": ([_c_i64, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_sz)],
                                            _c_int),
    "cg_lstm_weight_grads": ([_c_i64, _c_i32, _c_i32, _c_i32, _vp, _c_i64, _vp, _c_i64, _vp, _vp, _vp,
                              _vp, _vp, _c_sz, _vp], _c_int),
    "cg_bias_grad_workspace_bytes": ([_c_i64, _c_i32, ctypes.POINTER(_c_sz)], _c_int),
    "cg_bias_grad": ([_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _c_sz, _vp], _c_int),
    "cg_bias_act_forward": ([_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp], _c_int),
    "cg_bias_act_workspace_bytes": ([_c_i64, _c_i32, ctypes.POINTER(_c_sz)], _c_int),
    "cg_bias_act_backward": ([_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _c_i32, _vp, _c_sz, _vp],
                             _c_int),
    "cg_gemm_f32": ([_c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _c_i32, _vp, _c_i32, _vp, _c_i32,
                     _vp], _c_int),
    "cg_fourier_workspace_bytes": ([_c_i32, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_sz),
                                    ctypes.POINTER(_c_sz)], _c_int),
    "cg_fourier_forward": ([_c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp],
                           _c_int),
    "cg_fourier_backward": ([_c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_sz,
                             _vp], _c_int),
    "cg_lstm_cell_forward": ([_c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
                             _c_int),
    "cg_lstm_cell_backward": ([_c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
                              _c_int),
    "cg_lstm_hconv_supported": ([_vp, _c_i32, _c_i32, ctypes.POINTER(_c_i32)], _c_int),
    "cg_lstm_hconv_step": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                            _vp, _vp, _c_i64, _vp], _c_int),
    "cg_lstm_seq_supported": ([_vp, _c_i32, _c_i32, ctypes.POINTER(_c_i32)], _c_int),
    "cg_lstm_seq_workspace_bytes": ([_vp, _c_i32, ctypes.POINTER(_c_sz)], _c_int),
    "cg_lstm_seq_forward": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp,
                             _vp, _vp, _vp, _vp, _c_i64, _vp, _c_sz, _vp], _c_int),
    "cg_lstm_seq_status": ([_vp, _c_i32, _vp, ctypes.POINTER(_c_i32), _vp], _c_int),
    "cg_lstm_seq_fault": ([_vp, _c_i32, _c_i32, ctypes.POINTER(_c_i32)], _c_int),
    "cg_plan_set_seq_fault_test": ([_vp, _c_i32], _c_int),
    "cg_set_option": ([_c_i32, _c_i32], _c_int),
    "cg_get_option": ([_c_i32, ctypes.POINTER(_c_i32)], _c_int),
    "cg_dropout_forward": ([_vp, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64, _vp, _vp], _c_int),
    "cg_dropout_backward": ([_vp, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64, _vp, _vp], _c_int),
    "cg_clip_by_norm": ([_vp, ctypes.c_int64, ctypes.c_float, _vp, _vp], _c_int),
    "cg_lstm_seq_x_supported": ([_vp, _c_i32, _c_i32, _c_i32, ctypes.POINTER(_c_i32)], _c_int),
    "cg_lstm_seq_forward_x": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp,
                               _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _c_sz,
                               _vp], _c_int),
    "cg_lstm_bwd_step": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _c_i32, _vp,
                          _vp, _vp, _vp, _vp, _vp, _vp], _c_int),
    "cg_perm_gather": ([_vp, _vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp], _c_int),
    "cg_maxpool_forward": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp], _c_int),
    "cg_maxpool_backward": ([_vp, _vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp], _c_int),
    "cg_avgpool_forward": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp], _c_int),
    "cg_avgpool_backward": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp], _c_int),
    "cg_cheb_backward_adam": ([_vp, _c_i32, _c_i32, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp,
                               _vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                               _c_i32, ctypes.c_float, _vp, _c_sz, _vp], _c_int),
    "cg_adam_update": ([_vp, _vp, _vp, _vp, _c_i64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                        ctypes.c_float, _c_i32, ctypes.c_float, _vp], _c_int),
    "cg_sgd_update": ([_vp, _vp, _c_i64, ctypes.c_float, ctypes.c_float, _vp], _c_int),
    "cg_rmsprop_update": ([_vp, _vp, _vp, _vp, _c_i64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                           ctypes.c_float, ctypes.c_float, _vp], _c_int),
    "cg_comm_unique_id": ([ctypes.c_char_p], _c_int),
    "cg_comm_init": ([ctypes.POINTER(_vp), _c_int, _c_int, ctypes.c_char_p, _c_int], _c_int),
    "cg_allreduce_sum_f32": ([_vp, _vp, _c_sz, _vp], _c_int),
    "cg_comm_destroy": ([_vp], _c_int),
    "cg_comm_count": ([_vp, ctypes.POINTER(_c_int)], _c_int),
    "cg_comm_async_error": ([_vp, ctypes.POINTER(_c_int), _c_int], _c_int),
    # host-side coarsening: numpy arrays passed by pointer
    "cg_graclus_match_f32": ([_c_i64, _vp, _vp, _vp, _c_i32, _vp, _vp, _vp,
                              ctypes.POINTER(_c_i32)], _c_int),
    "cg_graclus_match_f64": ([_c_i64, _vp, _vp, _vp, _c_i32, _vp, _vp, _vp,
                              ctypes.POINTER(_c_i32)], _c_int),
    "cg_compute_perm": ([_c_i32, _vp, _vp, _vp, _c_i64, _vp], _c_int),
}

_lib = None


def header_symbols(path: str = HEADER_PATH):
    """Every function the public header declares (used by the ABI-export test)."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(cg_\w+)\s*\(", text, re.M)))


def lib():
    """Load (once) and return the ctypes handle.  Raises ImportError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built: run `make` (or __graft_entry__.build()) -- "
            "cnn_graph_amd has no CPU/PyTorch fallback for its HIP kernels")
    h = ctypes.CDLL(LIB_PATH)
    for name, (argtypes, restype) in _SIGNATURES.items():
        fn = getattr(h, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = h
    return h


def check(func_name: str, status: int):
    if status != CG_OK:
        msg = lib().cg_last_error()
        raise CGError(func_name, status, msg.decode() if msg else "")


def get_option(name: str) -> int:
    v = ctypes.c_int32()
    call("cg_get_option", OPTIONS[name], ctypes.byref(v))
    return v.value


def set_option(name: str, value: int) -> int:
    """Set a kernel-selection option (process-wide); returns the previous value."""
    old = get_option(name)
    call("cg_set_option", OPTIONS[name], int(value))
    return old


class options:
    """Context manager: ``with _lib.options(dw_direct=0): ...`` restores on exit."""

    def __init__(self, **kw):
        self.kw, self.saved = kw, {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.saved[k] = set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_option(k, v)
        return False


def call(func_name: str, *args):
    """Call a C-ABI function and raise CGError on a non-zero status."""
    status = getattr(lib(), func_name)(*args)
    check(func_name, status)
    return status
