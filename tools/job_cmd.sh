# r05n: host-buffer NTT copy-back through pinned pieces + 8 host threads (fresh vs resident outputs)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d ${O}_tl -o run --output-format csv -- \
  python3 tools/ntt_fresh_trace.py > ${O}_tl.log 2>&1 || exit 1
grep -E "fresh|resident" ${O}_tl.log
timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
