set -o pipefail
mkdir -p gpurun_out/r03/multirank
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_bench_contract.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/gpu_shard.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03/gpu_shard.log; exit 1; }
tail -2 gpurun_out/r03/gpu_shard.log
timeout -k 10 240 python -u tools/shard_overhead_nccl.py > gpurun_out/r03/shard_overhead_nccl2.txt 2>&1 || { echo SHARD_FAILED; tail -20 gpurun_out/r03/shard_overhead_nccl2.txt; exit 1; }
grep "E=" gpurun_out/r03/shard_overhead_nccl2.txt
for k in 1 8; do timeout -k 10 120 python -u tools/shard_host_breakdown.py 512 $k > gpurun_out/r03/shard_host_breakdown_k$k.txt 2>&1 || { echo BD_FAILED; tail gpurun_out/r03/shard_host_breakdown_k$k.txt; exit 1; }; grep "E=" gpurun_out/r03/shard_host_breakdown_k$k.txt; done
BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 48 --warmup 8 > gpurun_out/r03/multirank/merge2_k8.log 2>&1 || { echo MR_FAILED; tail -20 gpurun_out/r03/multirank/merge2_k8.log; exit 1; }
grep "^{" gpurun_out/r03/multirank/merge2_k8.log | cut -c1-600
