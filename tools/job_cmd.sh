# r05i: populate with transparent huge pages
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ntt_e2e_probe.py 24 || exit 1
