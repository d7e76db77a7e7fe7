# r05f: (1) host-buffer NTT into fresh outputs: np.zeros vs np.empty allocation inside the timing;
# (2) group FFT at 2^16 after the membership-test register fix, with its kernel breakdown
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ${O}_pfft -o run --output-format csv -- \
  python3 tools/fft_time.py 16 3 > ${O}_pfft.log 2>&1 || exit 1
cat ${O}_pfft.log | grep group
