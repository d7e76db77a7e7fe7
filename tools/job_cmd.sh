# r05za: level-1/1.5 sort chunk (entries staged in LDS per round): 4096 (in-tree) vs 8192 vs 16384
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
for v in base sc8k sc16k; do
  L=""; [ $v != base ] && L=variants/$v/libzkalgebra_gpu.so
  echo "== $v"
  for m in 20 23 24; do
    ZK_LIB_PATH=$L timeout -k 10 200 python3 tools/sweep_window.py bls12_381 $m || exit 1
  done
  ZK_LIB_PATH=$L timeout -k 10 200 python3 tools/sweep_window.py bn128 24 || exit 1
  ZK_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_$v -o run --output-format csv -- \
    python3 tools/sweep_window.py bls12_381 24 > ${O}_$v.log 2>&1 || exit 1
done
