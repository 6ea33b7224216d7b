"""Static check of the counted vector-memory waits in the device assembly (tools/check_vmcnt.py).

The fused MLP kernels (csrc/mlp.hip) and the v9 GEMM K loop (csrc/gemm9.hip) retire their LDS-DMAs with counted
``s_waitcnt vmcnt(N)``: correct only if at least N vector-memory instructions follow the DMA in the instruction stream
the compiler emitted, on every path.  These tests compile both sources to gfx950 assembly with the library's own flags
and check every marked wait (SV_VMWAIT) against its DMA group (SV_VMTAG) -- no GPU needed.  The negative cases pin that
the checker sees a short wait, a skipped issue on one path and a wait whose count relies on a branch-correlated path.
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_vmcnt as cv  # noqa: E402

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.timeout(900)
@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
def test_shipped_counted_waits_retire_their_dma():
    asm = cv.build_asm()
    failures, counted = [], {}
    for src, text in asm.items():
        res = cv.check_text(text)
        counted[src] = len(res)
        for kern, rows in res.items():
            for r in rows:
                if not r["ok"] or not r["known"]:
                    failures.append(f"{src} {kern[:80]} line {r['line']}: vmcnt({r['vmcnt']}) must retire "
                                    f"{r['target']}, min younger {r['younger_min']}")
    # every fused-MLP kernel (forward C=128/192/256/512 train + eval, the C=128 pair, the backward) and every v9
    # instantiation carries checked waits
    assert counted["mlp.hip"] >= 11, counted
    assert counted["gemm9.hip"] >= 40, counted
    assert not failures, "\n".join(failures)


_HEAD = """\t.type\tk,@function
k:
"""
_TAIL = """\ts_endpgm
.Lfunc_end0:
"""


def _kernel(body: str) -> dict:
    res = cv.check_text(_HEAD + body + _TAIL, jobs=1)
    return res.get("k", [])


def test_checker_counts_younger_instructions():
    ok = _kernel("""\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds
\t; svtag w
\tbuffer_load_dwordx4 v2, s[0:3], 0 offen
\tbuffer_store_dwordx4 v[4:7], v3, s[0:3], 0 offen
\ts_waitcnt vmcnt(2) ; svwait w:1
""")
    assert ok and all(r["ok"] for r in ok)
    short = _kernel("""\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds
\t; svtag w
\tbuffer_load_dwordx4 v2, s[0:3], 0 offen
\ts_waitcnt vmcnt(2) ; svwait w:1
""")
    assert short and not short[0]["ok"] and short[0]["younger_min"] == 1


def test_checker_sees_a_path_that_skips_the_younger_instructions():
    # the round-5 mlp_fwd_kernel shape: the next chunk's issue skipped on one path, the wait's count assumes it
    rows = _kernel("""\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds
\t; svtag w
\ts_cmp_lt_i32 s4, s5
\ts_cbranch_scc1 .LBB0_2
\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds
\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds
.LBB0_2:
\ts_waitcnt vmcnt(2) ; svwait w:1
""")
    assert rows and not rows[0]["ok"] and rows[0]["younger_min"] == 0


def test_checker_follows_mask_correlated_branches():
    # hipcc's pattern: s[0:1] = -1 / 0 on the two sides of a first branch, a second branch on it: exactly one of the
    # two issue blocks runs, so the wait is covered on every feasible path
    rows = _kernel("""\tbuffer_load_dwordx4 v1, s[8:11], 0 offen lds
\t; svtag w
\ts_cmp_ge_i32 s4, s5
\ts_mov_b64 s[0:1], -1
\ts_cbranch_scc0 .LBB0_2
\ts_mov_b64 s[0:1], 0
\tbuffer_load_dwordx4 v1, s[8:11], 0 offen lds
.LBB0_2:
\ts_andn2_b64 vcc, exec, s[0:1]
\ts_cbranch_vccnz .LBB0_3
\tbuffer_load_dwordx4 v1, s[8:11], 0 offen lds
.LBB0_3:
\ts_waitcnt vmcnt(1) ; svwait w:1
""")
    assert rows and rows[0]["ok"], rows


def test_checker_path_condition():
    # "w:1@e": only the paths on which group e was tagged after w's instance
    rows = _kernel("""\tbuffer_load_dwordx4 v1, s[8:11], 0 offen lds
\t; svtag w
\ts_cmp_lt_i32 s4, s5
\ts_cbranch_scc1 .LBB0_2
\tbuffer_store_dwordx4 v[4:7], v3, s[0:3], 0 offen
\tbuffer_store_dwordx4 v[4:7], v3, s[0:3], 0 offen
\t; svtag e
.LBB0_2:
\ts_waitcnt vmcnt(2) ; svwait w:1@e
""")
    assert rows and rows[0]["ok"], rows


@pytest.mark.timeout(900)
@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
def test_fused_mlp_bwd_ln_operands_consumed_below_their_wait():
    """The fused S1 MLP backward's LayerNorm operands (z / mean / rstd, group "zl") are read only below their own
    counted wait.  The unpinned cross-lane build (SV_MLPB_XLANE=3 SV_MLPB_PIN=0) -- the one measured to differ run to
    run in dz / dw (profiles/round6/r15_xlane_bisect) -- has its consumers hoisted above that wait, and the check
    must see it; the shipped build and the pinned cross-lane build must not."""
    shipped = cv.check_early_use_text(cv.build_asm(("mlp.hip",))["mlp.hip"])
    rows = [r for k, rs in shipped.items() if "mlpb128" in k for r in rs]
    assert rows and all(r["loads"] == 20 and r["wait"] is not None for r in rows), rows
    assert not any(r["uses"] for r in rows), [u for r in rows for u in r["uses"][:4]]
    pinned = cv.check_early_use_text(cv.build_asm(("mlp.hip",), ("-DSV_MLPB_XLANE=3",))["mlp.hip"])
    assert not any(r["uses"] for k, rs in pinned.items() if "mlpb128" in k for r in rs)
    bad = cv.check_early_use_text(cv.build_asm(("mlp.hip",), ("-DSV_MLPB_XLANE=3", "-DSV_MLPB_PIN=0"))["mlp.hip"])
    assert any(r["uses"] for k, rs in bad.items() if "mlpb128" in k for r in rs)


def test_early_use_check_on_a_synthetic_kernel():
    body = """\tbuffer_load_dwordx4 v[10:13], v1, s[0:3], 0 offen
\tbuffer_load_dwordx2 v[20:21], v2, s[4:7], 0 offen
\ts_nop 0
\tbuffer_load_dword v22, v3, s[8:11], 0 offen
\t; svtag zl
\tv_add_f32_e32 v30, v10, v31
{use}\ts_waitcnt vmcnt(0) ; svwait zl:1
\tv_mul_f32_e32 v32, v20, v22
"""
    clean = cv.check_early_use((_HEAD + body.format(use="") + _TAIL).splitlines())
    assert clean[0]["loads"] == 2 and not clean[0]["uses"]
    hoisted = cv.check_early_use((_HEAD + body.format(use="\tv_sub_f32_e32 v33, v21, v31\n") + _TAIL).splitlines())
    assert [ins for _, ins in hoisted[0]["uses"]] == ["v_sub_f32_e32 v33, v21, v31"]
