set -o pipefail
# tools/hop_latency.py at P = 2, 4, 8 on the one-GPU box (ranks sharing it),
# then the `widening` suite (tests outside the SURVEY 8 contract) once.
O=gpurun_out/r10j
mkdir -p $O
run() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2952$1 tools/hop_latency.py > $O/hop_p$1.json 2> $O/hop_p$1.err
}
run 2 4 && run 4 2 && run 8 1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m widening -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/widening_suite.txt 2>&1
