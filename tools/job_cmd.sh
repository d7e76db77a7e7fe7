# r05zj: lazy Fp2 squaring (ZK_FP2_LAZY) -- G2 MSM timings (before: r05zd 2.18 / 5.39 (BN128), 4.66 / 11.95 ms (BLS12-381))
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/g2_time.py || exit 1
