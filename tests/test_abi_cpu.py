"""C-ABI checks that need no GPU: the library loads, exports every symbol the
public header declares, and rejects bad arguments before touching the device."""
import ctypes

import numpy as np
import pytest

from cnn_graph_amd import _lib


def test_library_exports_every_header_symbol(built_lib):
    import os
    h = _lib.lib()
    public = _lib.header_symbols()
    testing = _lib.header_symbols(os.path.join(os.path.dirname(_lib.HEADER_PATH), "cheb_mi355_testing.h"))
    assert len(public) >= 19
    syms = sorted(set(public) | set(testing))
    missing = [s for s in syms if not hasattr(h, s)]
    assert missing == []
    assert set(syms) == set(_lib._SIGNATURES), "ctypes signatures out of sync with the headers"
    # the test-only fault hook is not part of the integration surface
    assert "cg_plan_set_seq_fault_test" not in public and testing == ["cg_plan_set_seq_fault_test"]


def test_version(built_lib):
    # 0.3.0 (round 6): ablation-only option values refused, the fault hook moved
    # to the testing header
    assert _lib.lib().cg_version() == 301


def test_release_library_refuses_ablation_only_options(built_lib):
    """The kernel alternatives that lost every A/B are in the ablation build
    only: the release library refuses their option values
    and does not contain their kernels."""
    h = _lib.lib()
    for name, v in (("dw_direct", 2), ("dw_direct", 3), ("dw_w2", 0), ("spmm_pw", 0), ("grp_pc", 0),
                    ("clen_dy", 0), ("clen_dy", 2), ("dw_x3", 2), ("gemm_x3", 2)):
        assert h.cg_set_option(_lib.OPTIONS[name], v) == _lib.CG_ERR_ARG, (name, v)
    for name, v in (("dw_direct", 0), ("dw_direct", 1), ("dw_w2", 1), ("spmm_pw", 1), ("grp_pc", 1),
                    ("clen_dy", 1), ("dw_x3", 0), ("dw_x3", 1), ("gemm_x3", 0), ("gemm_x3", 1)):
        assert h.cg_set_option(_lib.OPTIONS[name], v) == _lib.CG_OK, (name, v)
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    # the one-entry-per-access grp16 forward and the LDS-columns Clenshaw kernel
    for sym in (b"_ZN2cg12_GLOBAL__N_111k_grp16_fwdILi1ELb0EEEvNS0_10GrpFwdArgsE",
                b"_ZN2cg12_GLOBAL__N_110k_grp_clenILb0EEEvNS0_11GrpClenArgsE"):
        assert sym not in blob, sym


def test_release_library_has_no_ablation_hooks(built_lib):
    """The timing-ablation switches (outputs WRONG when set) exist only in the
    debug build (`make debug`); the shipping library must not export them."""
    h = _lib.lib()
    assert not hasattr(h, "cg_debug_set_flags")
    # no environment switches or env-driven fault injection either: kernel
    # choices go through cg_set_option, the hand-off fault test through the
    # plan-scoped cg_plan_set_seq_fault_test
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    for s in (b"getenv", b"CG_SEQ_INJECT_HANG", b"CG_SIDE_DW", b"CG_SEQ_V", b"k_lstm_seq2"):
        assert s not in blob, s


def test_options_roundtrip_and_validation(built_lib):
    h = _lib.lib()
    for name in _lib.OPTIONS:
        v = _lib.get_option(name)
        assert _lib.set_option(name, v) == v
    assert _lib.get_option("dw_waves") == 8 and _lib.get_option("dw_direct") == 1
    with _lib.options(dw_direct=0, seq_xpre=2):
        assert _lib.get_option("dw_direct") == 0 and _lib.get_option("seq_xpre") == 2
    assert _lib.get_option("dw_direct") == 1 and _lib.get_option("seq_xpre") == 1
    assert h.cg_set_option(99, 1) == _lib.CG_ERR_ARG
    assert h.cg_set_option(_lib.OPTIONS["dw_waves"], 5) == _lib.CG_ERR_ARG
    assert h.cg_set_option(_lib.OPTIONS["spmm_pw"], 2) == _lib.CG_ERR_ARG
    # the x-basis pre-pass: 0 in-loop, 1 one LDS launch (default), 2 per-order launches
    assert _lib.get_option("seq_xpre") == 1
    with _lib.options(seq_xpre=2):
        assert _lib.get_option("seq_xpre") == 2
    assert h.cg_set_option(_lib.OPTIONS["seq_xpre"], 3) == _lib.CG_ERR_ARG
    assert h.cg_get_option(0, None) == _lib.CG_ERR_ARG
    assert h.cg_plan_set_seq_fault_test(None, 1) == _lib.CG_ERR_ARG


def test_plan_variant_validation(built_lib):
    h = _lib.lib()
    assert h.cg_plan_set_variant(None, 0) == _lib.CG_ERR_ARG


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32).ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32).ctypes.data_as(ctypes.POINTER(ctypes.c_float))


@pytest.mark.parametrize("rowptr,col,msg", [
    ([0, 2, 3], [1, 0, 0], "not strictly increasing"),   # unsorted row 0
    ([0, 1, 2], [0, 5], "out of range"),                   # column >= M
    ([0, 2, 1], [0, 1], "rowptr"),                         # rowptr[M] != nnz / decreasing
])
def test_plan_create_rejects_bad_csr(built_lib, rowptr, col, msg):
    h = _lib.lib()
    rp, ci = np.array(rowptr, np.int32), np.array(col, np.int32)
    val = np.ones(len(ci), np.float32)
    out = ctypes.c_void_p()
    st = h.cg_plan_create(ctypes.byref(out), 0, 2, len(ci), _i32(rp), _i32(ci), _f32(val), None, None, None)
    assert st == _lib.CG_ERR_ARG
    assert msg in h.cg_last_error().decode()
    assert not out.value


def test_null_and_shape_errors(built_lib):
    h = _lib.lib()
    assert h.cg_plan_set_path(None, 0) == _lib.CG_ERR_ARG
    assert h.cg_cheb_forward(None, 1, 1, 1, 1, None, None, None, None, None, 0, None) == _lib.CG_ERR_ARG
    assert h.cg_maxpool_forward(None, 1, 6, 1, 4, None, None, None) == _lib.CG_ERR_ARG
    assert h.cg_adam_update(None, None, None, None, 1, 0.1, 0.9, 0.999, 1e-8, 0, 1.0, None) == _lib.CG_ERR_ARG
    assert h.cg_cheb_backward_adam(None, 1, 1, 2, 1, None, None, None, None, None, None, None,
                                   1e-3, 0.9, 0.999, 1e-8, 1, 1.0, None, 0, None) == _lib.CG_ERR_ARG
    assert "backward_adam" in h.cg_last_error().decode()
    # aliasing of dW / W / m / v is rejected before any device work
    p = ctypes.c_void_p(4096)
    q, r = ctypes.c_void_p(8192), ctypes.c_void_p(12288)
    assert h.cg_cheb_backward_adam(None, 1, 1, 2, 1, None, None, p, None, p, q, r,
                                   1e-3, 0.9, 0.999, 1e-8, 1, 1.0, None, 0, None) == _lib.CG_ERR_ARG
    assert "distinct" in h.cg_last_error().decode()
    with pytest.raises(_lib.CGError):
        _lib.call("cg_plan_set_path", None, 0)


def test_lstm_and_grad_entry_points_validate(built_lib):
    h = _lib.lib()
    sz = ctypes.c_size_t()
    assert h.cg_weight_grad_workspace_bytes(1000, 96, 128, ctypes.byref(sz)) == _lib.CG_OK
    assert sz.value >= 96 * 128 * 4
    assert h.cg_bias_grad_workspace_bytes(1000, 128, ctypes.byref(sz)) == _lib.CG_OK
    assert sz.value >= 128 * 4
    assert h.cg_weight_grad(0, 96, 128, None, None, None, 0, None, 0, None) == _lib.CG_ERR_ARG
    assert h.cg_bias_grad(10, 4, None, None, 0, None, 0, None) == _lib.CG_ERR_ARG
    # unknown gate set / null operands are rejected before any launch
    assert h.cg_lstm_cell_forward(4, 2, 7, 1, None, None, None, 1, 1, None, None) == _lib.CG_ERR_ARG
    assert "gate" in h.cg_last_error().decode()
    assert h.cg_lstm_cell_forward(4, 2, 0, None, None, None, None, None, None, None, None) == _lib.CG_ERR_ARG
    assert h.cg_lstm_cell_backward(4, 2, 0, None, None, None, None, None, None, None, None, None) == _lib.CG_ERR_ARG
    assert h.cg_lstm_cell_forward(1 << 30, 8, 0, 1, None, None, None, 1, 1, None, None) == _lib.CG_ERR_ARG
    assert "2^31" in h.cg_last_error().decode()


def test_stack_merge_and_loss_ema_entry_points_validate(built_lib):
    """stack_num > 1 pieces and the loss moving average reject bad arguments
    before any device work (no GPU needed)."""
    h = _lib.lib()
    p, q, r = ctypes.c_void_p(4096), ctypes.c_void_p(8192), ctypes.c_void_p(12288)
    assert h.cg_slice_channels(p, 10, 16, 12, 17, q, None) == _lib.CG_ERR_ARG
    assert "[12, 17)" in h.cg_last_error().decode()
    assert h.cg_slice_channels(p, 10, 16, 4, 4, q, None) == _lib.CG_ERR_ARG
    assert h.cg_stack_merge_forward(2, 10, 2, p, q, 0, p, None) == _lib.CG_ERR_ARG
    assert "alias" in h.cg_last_error().decode()
    assert h.cg_stack_merge_backward(2, 10, 2, p, q, r, None, None, None) == _lib.CG_ERR_ARG
    assert h.cg_stack_merge_backward(2, 10, 2, p, q, r, p, None, None) == _lib.CG_ERR_ARG
    assert h.cg_mse_loss_ema(p, q, 10, r, None, None, 0.9, None, 0, None) == _lib.CG_ERR_ARG
    assert h.cg_mse_loss_ema(p, q, 10, r, None, r, 1.5, None, 0, None) == _lib.CG_ERR_ARG


def test_basis_layout_entry_points_validate(built_lib):
    """Orders-layout entry points reject a null plan / unknown layout before any
    device work (no GPU needed)."""
    h = _lib.lib()
    n = ctypes.c_int64()
    assert h.cg_cheb_basis_elems(None, 1, 1, 2, 1, _lib.CG_BASIS_ORDERS, ctypes.byref(n)) == _lib.CG_ERR_ARG
    assert h.cg_cheb_forward_layout(None, 1, 1, 2, 1, None, None, None, 0, _lib.CG_BASIS_ORDERS,
                                    None, None, None, 0, None) == _lib.CG_ERR_ARG
    assert h.cg_cheb_backward_layout(None, 1, 1, 2, 1, None, None, 0, _lib.CG_BASIS_ORDERS, None,
                                     None, None, 0, None, None, None, 0, None) == _lib.CG_ERR_ARG
    assert h.cg_cheb_backward_adam_layout(None, 1, 1, 2, 1, _lib.CG_BASIS_ORDERS, None, None, None,
                                          None, None, None, None, 1e-3, 0.9, 0.999, 1e-8, 1, 1.0,
                                          None, 0, None) == _lib.CG_ERR_ARG
    assert h.cg_cheb_backward_layout(None, 1, 1, 2, 1, None, None, 7, _lib.CG_BASIS_ORDERS, None,
                                     None, None, 0, None, None, None, 0, None) == _lib.CG_ERR_ARG
    assert "activation" in h.cg_last_error().decode()


def test_forward_adam_validates(built_lib):
    """cg_cheb_forward_adam rejects missing operands and aliased outputs before
    any device work."""
    h = _lib.lib()
    p, q, r = ctypes.c_void_p(4096), ctypes.c_void_p(8192), ctypes.c_void_p(12288)
    g, m, v = ctypes.c_void_p(16384), ctypes.c_void_p(20480), ctypes.c_void_p(24576)
    y = ctypes.c_void_p(28672)
    assert h.cg_cheb_forward_adam(None, 1, 1, 2, 1, None, None, None, None, None, 1e-3, 0.9, 0.999,
                                  1e-8, 1, 1.0, None, None, None, 0, None, None, None, 0,
                                  None) == _lib.CG_ERR_ARG
    # W_out aliasing W
    assert h.cg_cheb_forward_adam(None, 1, 1, 2, 1, None, p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1,
                                  1.0, p, q, r, 0, None, y, None, 0, None) == _lib.CG_ERR_ARG
    assert "alias" in h.cg_last_error().decode()
    # m_out == v_out
    assert h.cg_cheb_forward_adam(None, 1, 1, 2, 1, None, p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1,
                                  1.0, q, r, r, 0, None, y, None, 0, None) == _lib.CG_ERR_ARG
    assert "distinct" in h.cg_last_error().decode()


def test_header_enums_match_the_binding(built_lib):
    """The ctypes binding's constants are the header's (basis layouts, paths,
    variants, activations, status codes)."""
    import re
    from cnn_graph_amd import _lib
    text = open(_lib.HEADER_PATH).read()
    consts = {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(CG_[A-Z_]+)\s*=\s*(-?\d+)", text)}
    for name in ("CG_BASIS_ROWS", "CG_BASIS_ORDERS", "CG_BASIS_PLANES", "CG_PATH_AUTO",
                 "CG_PATH_RESIDENT", "CG_PATH_STREAM", "CG_ACT_NONE", "CG_ACT_RELU"):
        assert name in consts, name
        assert getattr(_lib, name) == consts[name], name
    assert _lib.BASIS_LAYOUTS == {"rows": consts["CG_BASIS_ROWS"], "orders": consts["CG_BASIS_ORDERS"],
                                  "planes": consts["CG_BASIS_PLANES"]}


def test_update_rule_validation(built_lib):
    h = _lib.lib()
    assert h.cg_sgd_update(None, None, 4, 0.1, 1.0, None) == _lib.CG_ERR_ARG
    assert h.cg_sgd_update(None, None, 0, 0.1, 1.0, None) == _lib.CG_ERR_ARG
    assert h.cg_rmsprop_update(None, None, None, None, 4, 0.1, 0.9, 0.0, 1e-10, 1.0, None) == _lib.CG_ERR_ARG
