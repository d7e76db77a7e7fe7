# scratch commands of the current GPU experiment (run by tools/gpu_job.sh step "cmd")
# host arithmetic of finish_host on the box's CPU (ADX products when CPUID has them)
tools/microbench/host_chain
