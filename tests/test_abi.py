"""CPU: the C-ABI library loads and exports every symbol include/sv_kernels.h declares; argument
validation fails loudly (no GPU needed for the error paths)."""

import ctypes

from spine_vision_amd import native as nv


def test_every_header_symbol_exported():
    L = nv.lib()
    syms = nv.header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(nv._SIGS), set(syms) ^ set(nv._SIGS)


def test_version_and_target():
    L = nv.lib()
    assert L.sv_version() >= 1
    assert L.sv_build_target().decode() == "gfx950"


def test_invalid_args_report_error():
    L = nv.lib()
    d = nv.GemmDesc()  # all-null descriptor
    d.M = d.N = d.K = 8
    rc = L.sv_gemm(ctypes.byref(d), None)
    assert rc == 1
    assert "null" in L.sv_last_error_string().decode()
    rc = L.sv_layernorm_fwd(None, 0, None, None, None, 0, None, None, 10, 128, 1e-6, None)
    assert rc == 1


def test_nparts_queries():
    assert nv.value("sv_layernorm_bwd_nparts", 1000, 128) >= 1
    assert nv.value("sv_dwconv7_bwd_weight_nparts", 32, 128, 128, 128) >= 1
    assert nv.value("sv_sqnorm_nparts", 10_000_000) >= 1
