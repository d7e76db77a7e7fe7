# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
export ZK_LIB_PATH=$PWD/variants/onechain/libzkalgebra_gpu.so
timeout 300 python -u -m pytest tests/test_gpu_msm.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -3
timeout 300 python -u tools/sweep_window.py phases
