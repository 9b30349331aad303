"""CPU: libhgd.so loads and exports every symbol include/hgd.h declares (no compute calls)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(hgd_\w+)\s*\(", text))
    return sorted(names)


def test_header_declares_api():
    syms = header_symbols()
    assert "hgd_spmm" in syms and "hgd_sort_perm" in syms and len(syms) >= 20


def test_library_exports_every_header_symbol():
    import ctypes
    from hypergraph_diffusion_for_recommendation_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.fail(f"libhgd.so missing at {_native.LIB_PATH}: run __graft_entry__.build()")
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, f"not exported: {missing}"


def test_binding_table_covers_header():
    from hypergraph_diffusion_for_recommendation_amd import _native
    assert sorted(_native.symbols()) == header_symbols()


def test_load_binds_and_reports_version():
    from hypergraph_diffusion_for_recommendation_amd import _native
    lib = _native.load()
    assert lib.hgd_version() >= 100
    assert lib.hgd_get_last_error_string() == b""


def test_product_path_has_no_cpu_fallback():
    """spmm on a CPU tensor raises instead of silently computing on the host."""
    import torch
    from hypergraph_diffusion_for_recommendation_amd.incidence import CSR, spmm_csr
    csr = CSR(torch.zeros(2, dtype=torch.int64), torch.zeros(0, dtype=torch.int32), 1, 1,
              split_threshold=0)
    with pytest.raises(RuntimeError):
        spmm_csr(csr, torch.ones(1, 4))


def test_masked_row_gemm_rejects_forward_epilogues():
    """Argument validation only (returns before any HIP call): the masked (backward-data) form
    of hgd_gemm_rows takes none of the forward epilogues its kernel no longer carries (the
    output dropout is allowed: it is the backward of an input dropout fused into the forward)."""
    import ctypes
    from hypergraph_diffusion_for_recommendation_amd import _native
    lib = _native.load()
    d = _native.GemmRowsDesc()
    d.A, d.lda, d.relu_mask, d.ldm = 16, 64, 16, 64
    d.B, d.bsk, d.bsn, d.Y, d.ldy = 16, 64, 1, 16, 64
    d.rows, d.K, d.N = 1000, 64, 64
    d.res, d.ldres, d.Y2, d.ldy2 = 16, 64, 16, 64
    arr = (_native.GemmRowsDesc * 1)(d)
    assert lib.hgd_gemm_rows(arr, 1, None) == 1  # HGD_ERR_INVALID_ARG
    assert b"relu_mask excludes" in lib.hgd_get_last_error_string()


def test_package_never_imports_oracle():
    pkg = os.path.join(ROOT, "hypergraph_diffusion_for_recommendation_amd")
    for path in glob.glob(os.path.join(pkg, "**", "*.py"), recursive=True):
        src = open(path).read()
        assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, flags=re.M), path


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors (SplitPlan, RowEpilogue, IncidenceView, the grouped GEMM descriptors)
    have the header's size and field offsets."""
    import shutil
    import subprocess
    from hypergraph_diffusion_for_recommendation_amd import _native
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"hgd_split_plan": _native.SplitPlan, "hgd_row_epilogue": _native.RowEpilogue,
               "hgd_incidence_view": _native.IncidenceView,
               "hgd_gemm_rows_desc": _native.GemmRowsDesc, "hgd_gemm_tn_desc": _native.GemmTnDesc,
               "hgd_infonce_term": _native.InfonceTerm, "hgd_adam_tensor": _native.AdamTensor,
               "hgd_masked_sum": _native.MaskedSum}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hgd.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for cname, py in structs.items():
        assert got[(cname, "size")] == __import__("ctypes").sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_c_host_example_compiles_against_the_header(tmp_path):
    """include/hgd.h is valid C11 and every call of the examples/ hosts (flat ABI and incidence
    objects + RCCL exchange) links against libhgd.so (compile + link only: no device here)."""
    if not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("ROCm headers not available")
    from tests._native_host import build
    for src in ("hgconv2_host.c", "conv2hop_objects.c"):
        exe = build(tmp_path / src[:-2], src)
        if exe is None:
            pytest.skip("gcc not available")
        assert os.path.exists(exe)


def test_tuning_keys_validate_their_values():
    """hgd_set_tuning (host-side globals, no device work): every documented key takes its
    documented values, rejects others with HGD_ERR_INVALID_ARG, and the defaults restore."""
    from hypergraph_diffusion_for_recommendation_amd import _native
    lib = _native.load()
    good = {1: [8, 16], 2: [0, 1, 8, 9], 3: [0, 64, 128, 256], 4: [0, 64, 8192],
            5: [0, 64, 65536], 6: [0, 1], 7: [0, 64, 128], 8: [0, 1, 2], 9: [0, 1, 2, 3]}
    bad = {2: [3], 3: [32], 4: [63], 5: [65], 6: [2], 7: [32], 8: [3, -1], 9: [4, -1]}
    defaults = {1: 8, 2: 8, 3: 0, 4: 0, 5: 0, 6: 0, 7: 0, 8: 2, 9: 0}
    try:
        for key, vals in good.items():
            for v in vals:
                assert lib.hgd_set_tuning(key, v) == 0, (key, v)
        for key, vals in bad.items():
            for v in vals:
                assert lib.hgd_set_tuning(key, v) == 1, (key, v)
        assert lib.hgd_set_tuning(99, 0) == 1
    finally:
        for key, v in defaults.items():
            lib.hgd_set_tuning(key, v)
    # leave no error text behind for later tests that read hgd_get_last_error_string
    assert lib.hgd_set_tuning(8, 2) == 0
