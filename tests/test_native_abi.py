"""The C-ABI library builds, loads and exports every symbol include/ldsgnn.h
declares (no GPU needed: no compute calls)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ldsgnn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lds_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_hot_path():
    syms = declared_symbols()
    for s in ["lds_sample_bitmask", "lds_spmm_norm", "lds_theta_grad", "lds_sgd_clamp", "lds_dropout"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    import ldsgnn._native as nat
    lib = ctypes.CDLL(nat.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_bindings_cover_header():
    import ldsgnn._native as nat
    bound = set(nat.SIGNATURES) | {"lds_error_string"}
    assert set(declared_symbols()) <= bound


def test_abi_version_and_host_helpers():
    import ldsgnn._native as nat
    assert nat.lib.lds_abi_version() == nat.ABI_VERSION
    assert nat.lib.lds_bitmask_words(1) == 2
    assert nat.lib.lds_bitmask_words(128) == 2
    assert nat.lib.lds_bitmask_words(129) == 4
    assert nat.lib.lds_error_string(0).decode()


def test_argument_errors_need_no_gpu():
    import ldsgnn._native as nat
    # invalid arguments are rejected before any launch (hipErrorInvalidValue = 1)
    assert nat.lib.lds_spmm_norm(None, None, None, 0, None, 0, 0, None, 0, 0, None) == 1
    assert nat.lib.lds_theta_grad(None, None, 0, 0, None, 0, 0, None, 0, None, 0, None) == 1


def test_product_path_refuses_cpu_tensors():
    import pytest
    import torch
    from ldsgnn import ops
    with pytest.raises(RuntimeError, match="HIP device"):
        ops.sample_graph_from_triu(torch.rand(6), 3)


def test_theta_grad_form_selection_needs_no_gpu():
    """The θ-grad assembly form is host-side state (lds_theta_grad_set_form):
    default split bf16, every named form round-trips, out-of-range codes are
    rejected."""
    import ctypes as C

    import ldsgnn._native as nat
    from ldsgnn import ops
    assert ops.theta_grad_form() == "bf16x3"
    try:
        for name in ops.THETA_GRAD_FORMS:
            ops.theta_grad_form(name)
            assert ops.theta_grad_form() == name
    finally:
        ops.theta_grad_form("bf16x3")
    prev = C.c_int(-7)
    assert nat.lib.lds_theta_grad_set_form(len(ops.THETA_GRAD_FORMS), C.byref(prev)) == 1
    assert nat.lib.lds_theta_grad_set_form(-1, C.byref(prev)) == 0 and prev.value == 1
