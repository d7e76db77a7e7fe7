set -o pipefail
cd $GRAFT_REPO_ROOT
for ch in 16 32 48 64 96 128; do
  ZK_MSM_CH=$ch ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 20 0 2>&1 | tail -2 | head -1 | sed "s/^/CH=$ch /" || exit 1
done
for ch in 32 64 128; do
  ZK_MSM_CH=$ch ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py bls12_381 23 0 2>&1 | tail -2 | head -1 | sed "s/^/2^23 CH=$ch /" || exit 1
done
