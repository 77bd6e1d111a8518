set -o pipefail
mkdir -p gpurun_out/r03/multirank
timeout -k 10 240 python -u tools/shard_overhead_nccl.py > gpurun_out/r03/shard_overhead_nccl.txt 2>&1 || { echo SHARD_FAILED; tail -20 gpurun_out/r03/shard_overhead_nccl.txt; exit 1; }
cat gpurun_out/r03/shard_overhead_nccl.txt | grep -v amdgpu.ids
BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/r03/multirank/merge2.log 2>&1 || { echo MR_FAILED; tail -20 gpurun_out/r03/multirank/merge2.log; exit 1; }
tail -c 600 gpurun_out/r03/multirank/merge2.log
