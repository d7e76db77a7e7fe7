# r05n: host-buffer NTT copy-back through pinned pieces + 8 host threads (fresh vs resident outputs)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d ${O}_tl -o run --output-format csv -- \
  python3 tools/ntt_fresh_trace.py > ${O}_tl.log 2>&1 || exit 1
grep -E "fresh|resident" ${O}_tl.log
timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
# (2) Y sums at BLS12-381 2^20 (c = 16): k_ysum2 vs k_ysum3 at 4 / 8 / 16 buckets per lane
for y in 0 1; do
  for q in 4 8 16; do
    echo "== 2^20 ZK_YSUM3=$y ZK_YSUM_QY=$q"
    ZK_YSUM3=$y ZK_YSUM_QY=$q timeout -k 10 120 python3 tools/sweep_window.py bls12_381 20 16 || exit 1
  done
done
