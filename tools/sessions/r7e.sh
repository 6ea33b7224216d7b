#!/bin/bash
# round 4: in-kernel split-K fold (bitwise tests + step A/B) and the depthwise XCD-contiguous order (PMC traffic A/B)
set -u
O=gpurun_out/r7e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -rP --timeout 200 --timeout-method thread tests/test_gemm_family_gpu.py -k "fold" > $O/fold.log 2>&1
rc=$?; echo "fold tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for f in 1 0; do
    SV_INKERNEL_FOLD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_fold${f}_$i.json 2>>$O/bench.err || exit $?
  done
done
echo "bench done"
for x in 1 0; do
  SV_DW_XCD=$x timeout -k 10 120 python tools/dw_bench.py --iters 20 > $O/dw_xcd$x.txt 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && SV_DW_XCD=$x timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_dw_xcd${x}_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/dw_bench.py --stages S1,S3 --iters 2 > $GRAFT_REPO_ROOT/$O/pmc_dw_xcd${x}_$c.log 2>&1) || exit $?
  done
done
echo "dw done"
