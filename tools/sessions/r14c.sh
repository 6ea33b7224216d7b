#!/bin/bash
# round 6: the block weight gradients' grid target (SV_CNX_WGRAD_WGS 256 = whole chip, the default since round 4) against
# half the chip, now that the depthwise backward-data runs on the matrix cores with ~40 KB of LDS per workgroup (it cannot
# share a CU with a 128-160 KB weight-gradient workgroup), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r14c}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
i=0
for f in 128 256 128 256 192; do
  i=$((i+1))
  SV_CNX_WGRAD_WGS=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${f}_$i.json 2> $O/bench_$f.err || { tail -5 $O/bench_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${f}_$i.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('wgrad_wgs=$f train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'], 'dw_bwd_data', k['dw_bwd_data']['avg_launch_us'], 'fc2_dgrad', k['fc2_dgrad']['avg_launch_us'], 'wgrad', k['wgrad']['avg_launch_us'])"
done
