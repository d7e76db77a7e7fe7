# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
set -e
timeout 120 tools/microbench/copy_bw
