"""HBM traffic per launch of a kernel from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; kB).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts exactly half the bytes of a
wide (16 B/lane) coalesced streaming read -- the LDS-DMA loads of the GEMM are such reads -- so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores (the GEMM epilogue's stores).

    python tools/pmc_traffic.py <out_dir> <kernel substrings, '|'-separated> <key> <config> [profiles/traffic.json]

<config> = backbone/image/bs<batch>/<precision> of the bench run the passes profiled (bench.py looks the
bytes up under exactly that key and reports null otherwise).  A kernel CLASS (the forward GEMMs: fc1 on v3, fc2 on v2, downsample on v3) is matched by several
substrings; the per-launch figure is the mean over every matched launch, like bench.py's probe.
"""
import csv
import json
import os
import sys

out, pat, key, cfg = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
pats = pat.split("|")
dst = sys.argv[5] if len(sys.argv) > 5 else "profiles/traffic.json"


def per_launch(counter):
    path = os.path.join(out, f"pmc_{counter}", "run_counter_collection.csv")
    vals = {}
    for r in csv.DictReader(open(path)):
        if any(p_ in r["Kernel_Name"] for p_ in pats) and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sum(vals.values()) / max(len(vals), 1), len(vals)


fetch, nf = per_launch("FETCH_SIZE")
write, nw = per_launch("WRITE_SIZE")
traffic = (2.0 * fetch + write) * 1024.0
root = json.load(open(dst)) if os.path.exists(dst) else {}
data = root.setdefault("configs", {}).setdefault(cfg, {})
data[f"{key}_bytes_per_launch"] = round(traffic)
data[f"{key}_detail"] = {"kernel_match": pat, "launches": [nf, nw], "FETCH_SIZE_kB_raw": round(fetch, 1),
                         "WRITE_SIZE_kB": round(write, 1), "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024",
                         "source": out}
json.dump(root, open(dst, "w"), indent=1)
print(json.dumps(data, indent=1))
