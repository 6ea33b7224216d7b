"""The cross-lane form of the fused S1 MLP backward (csrc/mlp.hip ``SV_MLPB_XLANE=3``: the LayerNorm epilogue's
butterflies from permlane / DPP instead of ds_bpermute), with its LayerNorm operands pinned below their counted wait
(``SV_MLPB_PIN``, default), is bitwise run to run at ConvNeXt-base S1's M = 524288 (DESIGN
"Round 6").  Without the pin that build differed run to run in dz / dw (profiles/round6/r15_xlane_bisect).

The A/B library comes from ``tools/build_xlane_bisect.sh`` (``XL=3``: spine-vision_amd/libsv_kernels_xl3.so, linked
from the in-tree objects); the check runs tools/mlp_bwd_diag.py in a child process bound to it through SV_LIB_PATH,
three launches of the fused and the three-kernel path each."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "spine-vision_amd", "libsv_kernels_xl3.so")

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_cross_lane_fused_mlp_bwd_is_bitwise_run_to_run():
    if not os.path.exists(LIB):
        pytest.skip("A/B library absent (tools/build_xlane_bisect.sh with XL=3 builds it)")
    env = dict(os.environ, SV_LIB_PATH=LIB)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "mlp_bwd_diag.py"), "524288", "524288",
                        "524288"], env=env, capture_output=True, text=True, timeout=270)
    assert r.returncode == 0, r.stderr[-2000:]
    fused = [ln for ln in r.stdout.splitlines() if "fused deterministic" in ln and "unfused" not in ln]
    # per launch: dh, dz, dw, db of two runs equal bit for bit
    assert len(fused) == 3 and all(ln.endswith("True True True True") for ln in fused), r.stdout
