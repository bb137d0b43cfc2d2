set -o pipefail
# Synchronous run() latency of the plan-kernel ring at P = 2 (processes on
# the box's GPU) against the hardware queues per process.
O=gpurun_out/r10r
mkdir -p $O
for q in 1 2 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$q tools/hop_latency.py --sizes 1024,1048576 --engines plan_kernel > $O/p2_q$q.json 2> $O/p2_q$q.err || exit 1
done
