set -o pipefail
mkdir -p gpurun_out/r03
BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r03/bench_2rank_gloo.log 2>&1 || { echo BENCH2_FAILED; tail -30 gpurun_out/r03/bench_2rank_gloo.log; exit 1; }
grep "^{" gpurun_out/r03/bench_2rank_gloo.log | cut -c1-600
