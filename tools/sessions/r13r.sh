#!/bin/bash
# round 6: SQ split of the matrix-core depthwise weight gradient beside the VALU ring one (S3 / S1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13r}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d "$O/pmc_sq" -o run -- python3 "$ROOTDIR/tools/dw_bench.py" --stages S3,S1 --iters 2 > "$O/pmc_sq.log" 2>&1 || { tail -5 "$O/pmc_sq.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- python3 "$ROOTDIR/tools/dw_bench.py" --stages S3,S1 --iters 2 > "$O/pmc_fetch.log" 2>&1 || { tail -5 "$O/pmc_fetch.log"; exit 1; }
cd "$ROOTDIR"
python - $O/pmc_sq $O/pmc_fetch > $O/wgrad_sq.txt <<'PYEOF'
import collections, csv, glob, re, sys
for d in sys.argv[1:]:
    v = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            if "wgrad" not in nm:
                continue
            v[(nm[:60], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in sorted(v.items()):
        print(k[0], "grid", k[1])
        for c, xs in sorted(dd.items()):
            print(f"    {c:28s} {sum(xs) / len(xs):16.1f}")
PYEOF
cat $O/wgrad_sq.txt
