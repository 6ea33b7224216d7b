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
