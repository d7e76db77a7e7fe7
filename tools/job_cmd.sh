# r05c: Y sums at large windows -- k_ysum2 (one wave per SIMD) vs k_ysum3 (two waves, LDS
# prefetch), buckets per lane (QY), window sweep c = 16 / 18 / 20 at 2^23 and 2^24 (the per-GPU
# config-5 shards at N = 8 / 4), and the 2^23 / 2^26 kernel breakdowns under rocprof
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
for lg in 23 24; do
  for y in 0 1; do
    echo "== 2^$lg ZK_YSUM3=$y"
    ZK_YSUM3=$y timeout -k 10 120 python3 tools/sweep_window.py bls12_381 $lg 16 18 20 || exit 1
  done
  for q in 32 64; do
    echo "== 2^$lg ZK_YSUM3=1 ZK_YSUM_QY=$q"
    ZK_YSUM3=1 ZK_YSUM_QY=$q timeout -k 10 120 python3 tools/sweep_window.py bls12_381 $lg 20 || exit 1
  done
done
for y in 0 1; do
  ZK_YSUM3=$y timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ${O}_p23_y$y -o run --output-format csv -- \
    python3 tools/sweep_window.py bls12_381 23 20 > ${O}_p23_y$y.log 2>&1 || exit 1
done
ZK_YSUM3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${O}_p26_y1 -o run --output-format csv -- \
  python3 tools/sweep_window.py bls12_381 26 20 > ${O}_p26_y1.log 2>&1 || exit 1
echo "== 2^26 both"
for y in 0 1; do ZK_YSUM3=$y timeout -k 10 200 python3 tools/sweep_window.py bls12_381 26 20 || exit 1; done
