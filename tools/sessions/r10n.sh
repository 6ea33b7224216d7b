set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r10n
for d in 0 1 2 3; do
  L=""; [ $d != 0 ] && L=$PWD/spine-vision_amd/libsv_kernels_dwd$d.so
  echo "== variant $d"
  SV_LIB_PATH=$L timeout -k 10 120 python tools/dw_bench.py --stages S1,S3 --iters 30 || exit 1
done
