set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ch in 64 128 256; do
  for cfg in "bls12_381 23" "bls12_381 20" "bn128 22"; do
    echo "CH=$ch $cfg" >> gpurun_out/ch30.txt
    ZK_MSM_CH=$ch ZK_MSM_PROFILE=1 timeout -k 10 120 python tools/sweep_window.py $cfg 0 2>&1 | tail -2 >> gpurun_out/ch30.txt || exit 1
  done
done
echo ok
