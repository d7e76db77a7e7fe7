# r04s: split weights x copy mode (host-buffer MSM 2^20)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for rep in 1 2; do
  for m in 0 2; do
    for w in "2,3,4,4,3" "2,4,5,5" "2,3,4,5,2" "1,2,4,5,4" "3,4,4,3,2" "2,2,3,3,3,3"; do
      echo "== mode $m split $w"; ZK_COPY_MODE=$m ZK_MSM_SPLIT_W=$w timeout -k 10 120 python -u tools/e2e_probe.py bls12_381 20 15 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
