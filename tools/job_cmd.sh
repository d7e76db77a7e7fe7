# r04p: host-buffer MSM with the sort stream at the greatest priority (A/B ZK_SORT_PRIO=0), split weights under it
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for rep in 1 2 3; do
  echo "== prio default"; ZK_SORT_PRIO=0 timeout -k 10 120 python -u tools/e2e_probe.py bls12_381 20 20 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== prio high"; timeout -k 10 120 python -u tools/e2e_probe.py bls12_381 20 20 2>&1 | grep -v amdgpu.ids || exit 1
done
for w in "1,3,4,4,4" "2,3,4,4,3" "2,4,4,4,2" "1,2,3,3,3,2,2"; do
  echo "== high, split $w"; ZK_MSM_SPLIT_W=$w timeout -k 10 120 python -u tools/e2e_probe.py bls12_381 20 20 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r04p_trace -o run --output-format csv -- python3 tools/e2e_probe.py bls12_381 20 4 > gpurun_out/r04p_trace.log 2>&1 || exit 1
