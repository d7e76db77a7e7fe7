set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gputests8.log 2>&1; echo tests=$?
timeout -k 10 300 python bench.py > gpurun_out/bench8.json 2> gpurun_out/bench8.err; echo bench=$?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-ntt > gpurun_out/bench8_dist2.json 2> gpurun_out/bench8_dist2.err; echo dist=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ntt-steps 3 > gpurun_out/bench8p.json 2>gpurun_out/bench8p.err; echo prof=$?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc8a -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2>gpurun_out/pmc8a.err; echo pmca=$?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc8b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ntt-steps 2 > /dev/null 2>gpurun_out/pmc8b.err; echo pmcb=$?
