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


def _exported_lds_symbols(path):
    import shutil
    import subprocess
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return sorted({line.split()[-1] for line in out.splitlines() if line.split() and line.split()[-1].startswith("lds_")})


def test_library_exports_only_declared_entry_points():
    """libldsgnn.so exports exactly the header's entry points (plus
    lds_error_string): no ablation or variant entry point that returns wrong
    results ships in the product library (those live in the tools-only
    tools/variants/libldsgnn_variants.so)."""
    import ldsgnn._native as nat
    exported = set(_exported_lds_symbols(nat.LIB_PATH))
    assert exported == set(declared_symbols()) | {"lds_error_string"}, \
        sorted(exported ^ (set(declared_symbols()) | {"lds_error_string"}))
    assert "lds_spmm_dense_ablation" not in exported


def test_variants_library_is_tools_only():
    """The variants library (built by __graft_entry__.build() for the
    ablation tools) exports its tools entry points and nothing of the
    product's API."""
    import pytest
    path = os.path.join(ROOT, "tools", "variants", "libldsgnn_variants.so")
    if not os.path.exists(path):
        pytest.skip("tools/variants not built")
    assert _exported_lds_symbols(path) == ["lds_variants_spmm_dense", "lds_variants_spmm_dense_delayed",
                                          "lds_variants_spmm_dense_nt", "lds_variants_ws_bytes"]


def _kernel_metadata(lib_path, tmp_path):
    """{kernel symbol: (private segment bytes, VGPR spills)} of every gfx950
    code object in a built library (llvm-objdump --offloading + the
    code-object notes)."""
    import glob
    import shutil
    import subprocess
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-readelf")):
        import pytest
        pytest.skip("no llvm-readelf")
    lib = tmp_path / os.path.basename(lib_path)
    shutil.copy(lib_path, lib)
    subprocess.run([os.path.join(llvm, "llvm-objdump"), "--offloading", str(lib)], check=True, capture_output=True,
                   cwd=tmp_path)
    meta = {}
    for co in glob.glob(str(lib) + ".*gfx950"):
        notes = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
        for entry in notes.split("\n  - ")[1:]:
            kv = dict(re.findall(r"^\s+\.([a-z_]+):\s+(\S+)$", entry, flags=re.M))
            if "name" in kv and "private_segment_fixed_size" in kv:
                meta[kv["name"]] = (int(kv["private_segment_fixed_size"]), int(kv.get("vgpr_spill_count", 0)))
    return meta


def test_register_ring_kernels_have_no_scratch(tmp_path):
    """The spill-pass CSR-SpMM loads its column ring from inline asm
    (global_load_dwordx4 + counted s_waitcnt + a binding asm): if the compiler
    ever spilled or copied a ring register between the load and the wait, the
    kernel would read stale columns silently.  So every instantiation must
    compile without scratch (private segment 0, no VGPR spills); a compiler
    or flag change that adds spills fails here, at build time, instead of
    giving wrong sums."""
    import ldsgnn._native as nat
    meta = _kernel_metadata(nat.LIB_PATH, tmp_path)
    ring = {k: v for k, v in meta.items() if "csr_spill_agg_kernel" in k}
    assert len(ring) == 6, sorted(ring)  # 2 / 4 / 6 tiles × checked / unchecked
    for k, (private, spills) in ring.items():
        assert private == 0 and spills == 0, (k, private, spills)


def test_abi_version_matches_the_header():
    import ldsgnn._native as nat
    src = open(os.path.join(ROOT, "include", "ldsgnn.h")).read()
    m = re.search(r"#define LDS_ABI_VERSION (\d+)", src)
    assert m and int(m.group(1)) == nat.ABI_VERSION == nat.lib.lds_abi_version()


def test_xt_column_heads_are_128_wide():
    """ABI 18: lds_engine_xt_adam's `xthead` holds the first 128 row indices of
    every plan slot, zero past the column's end (the host builds it with
    LdsEngine._head_of); a one-wave column (<= 128 entries) then needs no index
    loads past its head."""
    import torch
    from ldsgnn.engine import LdsEngine
    g = torch.Generator().manual_seed(3)
    lens = torch.tensor([0, 1, 17, 64, 65, 128, 129, 300])
    p0 = torch.cat([torch.zeros(1, dtype=torch.long), lens.cumsum(0)[:-1]])
    rows = torch.randint(0, 5000, (int(lens.sum()),), generator=g, dtype=torch.int32)
    head = LdsEngine._head_of(p0, lens, rows, None, width=128)
    assert head.shape == (len(lens), 128) and head.dtype == torch.int32
    for c in range(len(lens)):
        k = min(int(lens[c]), 128)
        assert torch.equal(head[c, :k], rows[int(p0[c]):int(p0[c]) + k])
        assert int(head[c, k:].abs().sum()) == 0
