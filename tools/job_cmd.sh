# r05e: (1) where a host-buffer NTT into a fresh output spends its time (prefault on / off);
# (2) BLS12-381 MSM at c = 20 from 2^23 with the multi-load counting passes; 2^23 kernel breakdown
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
ZK_PREFAULT=0 timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
for lg in 20 23 24 26; do
  timeout -k 10 200 python3 tools/sweep_window.py bls12_381 $lg 0 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ${O}_p23 -o run --output-format csv -- \
  python3 tools/sweep_window.py bls12_381 23 20 > ${O}_p23.log 2>&1 || exit 1
# (3) group FFT at 2^12 / 2^16 (round-5 point routines, rolled membership chain) + kernel breakdown
timeout -k 10 120 python3 tools/fft_time.py 12 3 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ${O}_pfft -o run --output-format csv -- \
  python3 tools/fft_time.py 16 3 > ${O}_pfft.log 2>&1 || exit 1
