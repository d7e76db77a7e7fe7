# r05ze: lazy Jacobian doubling / cached addition in the BLS12-381 group FFT (ZK_FFT_LAZY)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
timeout -k 10 120 python3 tools/fft_time.py 16 3 || exit 1
timeout -k 10 200 python3 tools/fft_time.py 18 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d ${O}_trace -o run --output-format csv -- python3 tools/fft_time.py 16 1 > ${O}_trace.log 2>&1 || exit 1
