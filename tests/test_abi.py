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


def test_gemm_policy_validated_per_call():
    """The launch policy travels in the descriptor (sv_gemm_policy; there are no process-wide GEMM setters any
    more): an invalid policy is refused by argument validation, before anything is launched."""
    L = nv.lib()
    for name in ("sv_gemm_set_grid_cap", "sv_gemm_set_priority", "sv_gemm_set_workgroups_per_cu", "sv_gemm_set_impl"):
        assert not hasattr(L, name), name
    d = nv.GemmDesc()
    d.M = d.N = d.K = 64
    d.A = d.B = d.C = 1 << 20  # never dereferenced: validation fails first
    d.lda = d.ldb = d.ldc = 64
    d.a_kmajor = d.b_kmajor = 1
    d.a_dtype = d.b_dtype = d.compute = nv.SV_BF16
    d.policy = nv.policy(impl=5)
    assert L.sv_gemm(ctypes.byref(d), None) == 1
    assert "policy" in L.sv_last_error_string().decode()
    d.policy = nv.policy(wg_per_cu=3)
    assert L.sv_gemm(ctypes.byref(d), None) == 1
    assert "policy" in L.sv_last_error_string().decode()


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the header's structs have the C compiler's size and field offsets (gcc on the header)."""
    import os
    import subprocess

    structs = {"sv_gemm_desc": nv.GemmDesc, "sv_gemm_policy": nv.GemmPolicy, "sv_bn_ref": nv.BnRef,
               "sv_red_seg": nv.RedSeg, "sv_pack_seg": nv.PackSeg, "sv_conv_shape": nv.ConvShape,
               "sv_ctx_info": nv.CtxInfo}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sv_kernels.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-I", inc, "-D__HIP_PLATFORM_AMD__", str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, (cname, f)


def test_ctx_rejects_bad_devices():
    """sv_ctx_create validates the device ordinal (no GPU in the build container: every ordinal is out of range) and
    sv_ctx_destroy / sv_ctx_get_info refuse pointers that are not contexts."""
    L = nv.lib()
    h = ctypes.c_void_p()
    assert L.sv_ctx_create(-1, ctypes.byref(h)) == 1
    assert "no device" in L.sv_last_error_string().decode()
    assert L.sv_ctx_create(10**6, ctypes.byref(h)) == 1
    bogus = ctypes.c_void_p(16)
    assert L.sv_ctx_destroy(bogus) == 1
    assert L.sv_ctx_get_info(bogus, ctypes.byref(nv.CtxInfo())) == 1
