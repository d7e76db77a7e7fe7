# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
set -e
python bench.py --steps 3 --no-cpu-baseline --ntt-steps 2
