# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# r04c: host-buffer MSM after the copy-only stream / sort stream / weighted splits: phases + trace
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/e2e_probe.py bls12_381 20 20 --phases 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python -u tools/e2e_probe.py bn128 20 20 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/${TAG}_trace -o run --output-format csv -- \
  python3 tools/e2e_probe.py bls12_381 20 4 2>&1 | tail -1
