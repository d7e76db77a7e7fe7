# r05zd: Fp2 product as two shared-reduction pairs (ZK_FP2_LAZY=1) -- G2 MSM timings (exact form: r05w/r05zc)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/g2_time.py || exit 1
echo "== exact Fp2 product (variant fp2ex, ZK_FP2_LAZY=0)"
ZK_LIB_PATH=variants/fp2ex/libzkalgebra_gpu.so timeout -k 10 300 python3 tools/g2_time.py || exit 1
