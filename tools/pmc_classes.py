"""Per kernel CLASS summary of rocprofv3 --pmc passes over bench.py (one counter group per pass, each in
its own run): HBM traffic per launch, MFMA busy fraction and the effective shader clock.

    python tools/pmc_classes.py <out_dir> <config> [--traffic profiles/traffic.json] [--json out.json]

<out_dir> holds pass directories pmc_<NAME>/run_counter_collection.csv (tools/gpu_pmc.sh).  Definitions:
  * traffic = (2 * FETCH_SIZE + WRITE_SIZE) bytes per launch (gfx950: FETCH_SIZE reports half of a wide
    streaming read, MI355X_MICROARCH.md "HBM"); FETCH_SIZE and WRITE_SIZE come from separate passes;
  * MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the counter counts MFMA
    busy cycles summed over every SIMD, GRBM_GUI_ACTIVE the GPU-busy cycles summed over the 8 XCDs;
  * effective clock = GRBM_GUI_ACTIVE / 8 / launch duration, reported only over launches of >= 0.3 ms (it reads
    above the 2.4 GHz maximum on shorter ones, the guide's DVFS note; the in-kernel s_memtime clock is
    tools/clock_stamp.py's).
<config> (backbone/image/bs<batch>/<precision>) keys the traffic written into profiles/traffic.json.
"""
import argparse
import collections
import csv
import glob
import json
import os

# class -> alternatives; an alternative is a tuple of substrings that must all occur in the kernel name
CLASSES = {
    "wgrad": [("gemm9_kernel<false, false, 4,",), ("gemm3_kernel<false, false, 4,",)],
    "fc2_dgrad": [("gemm9_kernel<true, false, 6,",)],
    "dgrad": [("gemm9_kernel<true, false, 0,",)],  # keyed as bench.py's probe class (fc1 / downsample dgrad)
    "fwd": [("gemm9_kernel<true, true,",), ("gemm2_kernel<true, true",), ("gemm3_kernel<true, true",),
            ("gemm8_kernel<true, true",)],
    "dw_fwd": [("dwconv7_ring_kernel<", "false, false>")],
    "dw_bwd_data": [("dwconv7_ring_kernel<", "true, true>"), ("dwconv7_ring_kernel<", "true, false>")],
    "dw_wgrad": [("dwconv7_wgrad_ring_kernel<",)],
    "ln_bwd": [("ln_bwd_vec_kernel<",), ("ln_bwd_kernel<",)],
    "adamw": [("adamw_kernel",)],
    "mlp_fused": [("mlp_fwd_kernel<",), ("mlp128_kernel<",)],
    "mlp_bwd_fused": [("mlpb128_kernel",)],
    "fold": [("reduce_pair_kernel",), ("reduce_partials_kernel",), ("reduce_multi_kernel",),
             ("layerscale_reduce_kernel",)],
}


def klass(name):
    for c, alts in CLASSES.items():
        if any(all(s in name for s in alt) for alt in alts):
            return c
    return None


def load(out):
    """counter -> class -> {dispatch_id: (value, duration_ns)}"""
    res = collections.defaultdict(lambda: collections.defaultdict(dict))
    for path in glob.glob(os.path.join(out, "pmc_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            c = klass(r["Kernel_Name"])
            if c is None:
                continue
            d = res[r["Counter_Name"]][c]
            did = (path, r["Dispatch_Id"])
            v, dur = d.get(did, (0.0, 0))
            d[did] = (v + float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return res


def mean(d):
    return sum(v for v, _ in d.values()) / max(len(d), 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("config")
    ap.add_argument("--traffic", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = load(a.out)
    summary = {"source": a.out, "config": a.config, "classes": {}}
    for c in CLASSES:
        row = {}
        f, w = res.get("FETCH_SIZE", {}).get(c), res.get("WRITE_SIZE", {}).get(c)
        if f and w:
            row["launches"] = len(f)
            row["FETCH_SIZE_kB_raw"] = round(mean(f), 1)
            row["WRITE_SIZE_kB"] = round(mean(w), 1)
            row["traffic_bytes_per_launch"] = round((2.0 * mean(f) + mean(w)) * 1024.0)
        mb, ga = res.get("SQ_VALU_MFMA_BUSY_CYCLES", {}).get(c), res.get("GRBM_GUI_ACTIVE", {}).get(c)
        if mb and ga:
            busy, act = [], []
            clk = []
            for did, (gv, dur) in ga.items():
                if did in mb and gv > 0:
                    busy.append(mb[did][0] / (1024.0 * gv / 8.0))
                    if dur >= 300_000:  # the GRBM-derived clock is not evidence on dispatches under 0.3 ms
                        clk.append(gv / 8.0 / dur)
            row["mfma_busy_frac"] = round(sum(busy) / max(len(busy), 1), 4)
            if clk:
                row["eff_clock_ghz"] = round(sum(clk) / len(clk), 3)
            row["avg_launch_us_profiled"] = round(sum(dur for _, dur in ga.values()) / max(len(ga), 1) / 1e3, 2)
        sb = res.get("SQ_BUSY_CYCLES", {}).get(c)
        if sb and ga:
            row["sq_busy_frac"] = round(sum(sb[d][0] / (ga[d][0] / 8.0 * 32.0) for d in ga if d in sb and ga[d][0] > 0)
                                        / max(len(ga), 1), 4)
        if row:
            summary["classes"][c] = row
    print(json.dumps(summary, indent=1))
    if a.json:
        json.dump(summary, open(a.json, "w"), indent=1)
    if a.traffic:
        root = json.load(open(a.traffic)) if os.path.exists(a.traffic) else {}
        cfg = root.setdefault("configs", {}).setdefault(a.config, {})
        for c, row in summary["classes"].items():
            if "traffic_bytes_per_launch" in row:
                cfg[f"{c}_bytes_per_launch"] = row["traffic_bytes_per_launch"]
                cfg[f"{c}_detail"] = {"kernel_match": CLASSES[c], "launches": row["launches"],
                                      "FETCH_SIZE_kB_raw": row["FETCH_SIZE_kB_raw"], "WRITE_SIZE_kB": row["WRITE_SIZE_kB"],
                                      "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024", "source": a.out}
        json.dump(root, open(a.traffic, "w"), indent=1)


if __name__ == "__main__":
    main()
