# r05h: fresh-output NTT with the piecewise prefault / copy pipeline (prefault on / off)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
ZK_PREFAULT=0 timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
