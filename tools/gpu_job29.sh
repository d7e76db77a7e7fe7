set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "bls12_381 20" "bn128 20" "bls12_381 16" "bls12_381 23"; do
  ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py $cfg 0 >> gpurun_out/phases29.txt 2>&1 || exit 1
done
echo ok
