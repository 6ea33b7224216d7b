"""HBM-side traffic per dispatch class from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes (one counter per run):
traffic = 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE reports half of a wide streaming read,
MI355X_MICROARCH.md "HBM"), averaged per (kernel, grid) over the dispatches.

    python tools/pmc_traffic_by_kernel.py <fetch_pass_dir> <write_pass_dir> [name-substring]
"""
import collections
import csv
import glob
import re
import sys


def load(d, match):
    out = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            if match and match not in nm:
                continue
            out[(nm[:72], r["Grid_Size"])].append(float(r["Counter_Value"]))
    return out


match = sys.argv[3] if len(sys.argv) > 3 else ""
fe, wr = load(sys.argv[1], match), load(sys.argv[2], match)
for k in sorted(fe):
    f = sum(fe[k]) / len(fe[k])
    w = sum(wr.get(k, [0.0])) / max(1, len(wr.get(k, [])))
    print(f"{k[0]:72s} grid {k[1]:>9s}  traffic {(2 * f + w) / 1024:9.1f} MB  (2 x fetch {2 * f / 1024:9.1f}, write "
          f"{w / 1024:8.1f}; n={len(fe[k])})")
