# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
set -e
timeout 100 python tools/sweep_window.py bls12_381 14 6 7 8 9 10 11 12
timeout 100 python tools/sweep_window.py bls12_381 16 8 9 10 11 12 13 14
timeout 100 python tools/sweep_window.py bls12_381 18 11 12 13 14 15 16
timeout 100 python tools/sweep_window.py bn128 16 8 9 10 11 12 13 14
timeout 100 python tools/sweep_window.py bls12_381 12 5 6 7 8 9 10
