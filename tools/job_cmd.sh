# r05t: BN254 GLV stages at two waves per SIMD (222 VGPRs, no spill), operands not live across the chains
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
timeout -k 10 120 python3 tools/fft_time.py 16 3 || exit 1
timeout -k 10 200 python3 tools/fft_time.py 18 2 || exit 1
timeout -k 10 400 python3 tools/fft_time.py 20 1 || exit 1
