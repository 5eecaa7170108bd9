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
    assert nat.lib.lds_theta_grad(None, None, 0, 0, None, 0, 0, None, 0, None, 0, 1, None) == 1


def test_product_path_refuses_cpu_tensors():
    import pytest
    import torch
    from ldsgnn import ops
    with pytest.raises(RuntimeError, match="HIP device"):
        ops.sample_graph_from_triu(torch.rand(6), 3)


def test_theta_grad_form_is_a_per_call_argument():
    """The θ-grad assembly form is an argument of every lds_theta_grad* call
    (no library state: two engines with different forms in one process do not
    interfere).  ops.theta_grad_form() is the host-side default its callers
    pass; every named form round-trips, unknown names raise, and an
    out-of-range code is rejected by the library before any launch."""
    import pytest

    import ldsgnn._native as nat
    from ldsgnn import ops
    assert not hasattr(nat.lib, "lds_theta_grad_set_form") or "lds_theta_grad_set_form" not in nat.SIGNATURES
    assert ops.theta_grad_form() == "bf16x3" and ops.form_code() == 1
    try:
        for name, code in ops.THETA_GRAD_FORMS.items():
            ops.theta_grad_form(name)
            assert ops.theta_grad_form() == name and ops.form_code() == code
    finally:
        ops.theta_grad_form("bf16x3")
    with pytest.raises(ValueError):
        ops.theta_grad_form("bf16x4")
    # a valid call shape with form 11: hipErrorInvalidValue from the form check
    fake = 1 << 20  # never dereferenced: the argument checks run first
    assert nat.lib.lds_theta_grad(fake, fake, 8, 8, 0, 0, 0, 0, 16, fake, 0, 11, None) == 1
    assert nat.lib.lds_theta_grad(fake, fake, 8, 8, 0, 0, 0, 0, 16, fake, 0, -1, None) == 1


def test_graph_census_argument_errors_need_no_gpu():
    import ldsgnn._native as nat
    assert nat.lib.lds_graph_node_census(None, None, 0) == 1


def test_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirror of LdsBatch (ldsgnn._native) has
    the sizes and field offsets the C compiler gives include/ldsgnn.h."""
    import shutil
    import subprocess
    import ldsgnn._native as nat
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        import pytest
        pytest.skip("no C compiler")
    lines = []
    for st in (nat.LdsBatch,):
        lines.append(f'printf("{st.__name__} size %zu\\n", sizeof({st.__name__}));')
        for f, _ in st._fields_:
            lines.append(f'printf("{st.__name__} {f} %zu\\n", offsetof({st.__name__}, {f}));')
    src = tmp_path / "layout.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"ldsgnn.h\"\nint main(void){\n" +
                   "\n".join(lines) + "\nreturn 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(line.split()[:2]): int(line.split()[2]) for line in out if line}
    for st in (nat.LdsBatch,):
        assert got[(st.__name__, "size")] == ctypes.sizeof(st), st.__name__
        for f, _ in st._fields_:
            assert got[(st.__name__, f)] == getattr(st, f).offset, (st.__name__, f)
