set -o pipefail
cd $GRAFT_REPO_ROOT
for qy in 4 8 16 32; do
  ZK_MSM_QY=$qy ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/QY=$qy /" || exit 1
done
for qa in 2 4 8 16; do
  ZK_MSM_QA=$qa ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/QA=$qa /" || exit 1
done
for qy in 4 8 16; do
  ZK_MSM_QY=$qy ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bn128 20 0 2>&1 | tail -2 | head -1 | sed "s/^/BN QY=$qy /" || exit 1
done
