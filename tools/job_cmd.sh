# r05v: BN254 G2 k_accum at one wave per SIMD (349 VGPRs, no spill; variant g2bn1) vs two (256, 178 spilled); inversion chunk defaults
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
echo "== in-tree (ZK_ACCUM_WAVES20=2)"
timeout -k 10 300 python3 tools/g2_time.py bn128 || exit 1
echo "== g2bn1 (ZK_ACCUM_WAVES20=1)"
ZK_LIB_PATH=variants/g2bn1/libzkalgebra_gpu.so timeout -k 10 300 python3 tools/g2_time.py bn128 || exit 1
echo "== in-tree defaults: inversion chunks"
timeout -k 10 120 python3 tools/inv_probe.py || exit 1
