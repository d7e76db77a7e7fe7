# r05d: (1) group FFT A/B: round-5 doubling (D = 4XB, shared-reduction Y3, Karatsuba products;
# in-tree) vs the round-4 point routines (variants/fftold) at 2^12 / 2^16; (2) BLS12-381 MSM at
# c = 20 from 2^23 with the ballot-counted sub-bin split, vs ZK_SORT_SPLIT=0; kernel breakdown at 2^23
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
for m in 12 16; do
  for v in new old; do
    echo "== fft 2^$m $v"
    if [ $v = old ]; then L=variants/fftold/libzkalgebra_gpu.so; else L=; fi
    ZK_LIB_PATH=$L timeout -k 10 120 python3 tools/fft_time.py $m 3 || exit 1
  done
done
for lg in 23 24 26; do
  echo "== msm 2^$lg default window"
  timeout -k 10 200 python3 tools/sweep_window.py bls12_381 $lg 0 || exit 1
done
echo "== msm 2^23 ZK_SORT_SPLIT=0"
ZK_SORT_SPLIT=0 timeout -k 10 120 python3 tools/sweep_window.py bls12_381 23 20 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ${O}_p23 -o run --output-format csv -- \
  python3 tools/sweep_window.py bls12_381 23 20 > ${O}_p23.log 2>&1 || exit 1
