"""In-kernel shader clock of the v9 GEMM (MI355X_MICROARCH.md "DVFS give-back", item 6): run the
diagnostic library (tools/build_stamp.sh, -DSV_CLOCK_STAMPS) back to back for >= 2 s on random data, then
read every workgroup's s_memtime / s_memrealtime stamps of the LAST launch; clock = d(memtime) /
d(memrealtime) x 100 MHz (median over workgroups).  Diagnostic only: the product library has no stamps.

    SV_LIB_PATH=spine-vision_amd/libsv_kernels_stamp.so python tools/clock_stamp.py
"""

import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SV_LIB_PATH", os.path.join(ROOT, "spine-vision_amd", "libsv_kernels_stamp.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402
from spine_vision_amd import native as nv  # noqa: E402

PEAK_FLOP_PER_CLK = 256 * 4 * 1024  # CU x SIMD x dense bf16 FLOP/clk/SIMD


def main():
    dev = torch.device("cuda:0")
    L = nv.lib()
    fn = L.sv_diag_clock_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    M, C = 32768, 512  # ConvNeXt-base S3 at bs32
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    dh = torch.randn(M, 4 * C, device=dev, generator=g).to(bf)
    w1 = (torch.randn(4 * C, C, device=dev, generator=g) * 0.05).to(bf)
    y = torch.randn(M, C, device=dev, generator=g).to(bf)
    b1 = torch.zeros(4 * C, device=dev)
    dy = torch.empty(M, C, device=dev, dtype=bf)
    outh = torch.empty(M, 4 * C, device=dev, dtype=bf)
    outa = torch.empty_like(outh)
    cases = {
        "fc1_dgrad (K 2048, plain store)": (lambda: K.linear_dgrad(dh, w1, out=dy), 2.0 * M * C * 4 * C),
        "fc1_fwd (K 512, GELU dual)": (lambda: K.linear_fwd(y, w1, out=outh, out2=outa, bias=b1,
                                                            epilogue=nv.SV_EPI_BIAS_GELU_DUAL), 2.0 * M * C * 4 * C),
    }
    res = {}
    for name, (run, flops) in cases.items():
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        while time.perf_counter() - t0 < 2.5:
            for _ in range(50):
                run()
            n += 50
            torch.cuda.synchronize()
        ev1.record()
        torch.cuda.synchronize()
        us = ev0.elapsed_time(ev1) * 1e3 / n
        buf = (ctypes.c_ulonglong * (1024 * 4))()
        assert fn(buf, 1024) == 0
        st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 4).astype(np.float64)
        ok = st[:, 3] > st[:, 1]
        st = st[ok]
        clk = (st[:, 2] - st[:, 0]) / (st[:, 3] - st[:, 1]) * 100e6
        ghz = float(np.median(clk)) / 1e9
        tf = flops / (us * 1e-6) / 1e12
        bound = PEAK_FLOP_PER_CLK * ghz * 1e9 / 1e12
        res[name] = {"launches": n, "avg_us": round(us, 2), "tflops": round(tf, 1), "workgroups": int(ok.sum()),
                     "clock_ghz_median": round(ghz, 3), "clock_ghz_min": round(float(clk.min()) / 1e9, 3),
                     "clock_ghz_max": round(float(clk.max()) / 1e9, 3),
                     "dense_bf16_bound_at_this_clock_tflops": round(bound, 1),
                     "frac_of_clock_bound": round(tf / bound, 4), "frac_of_2516_peak": round(tf / 2516.6, 4)}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps({"clock_stamps": res}))


if __name__ == "__main__":
    main()
