# r05y: one-group sort beside the point conversion (device-resident, from 2^18) + BN128 two-group sort-ahead
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for m in 20 24; do
  echo "== bls 2^$m off"; ZK_MSM_AHEAD_MIN=0 timeout -k 10 200 python3 tools/sweep_window.py bls12_381 $m || exit 1
  echo "== bls 2^$m default"; timeout -k 10 200 python3 tools/sweep_window.py bls12_381 $m || exit 1
done
echo "== bn 2^24 default"; timeout -k 10 200 python3 tools/sweep_window.py bn128 24 || exit 1
