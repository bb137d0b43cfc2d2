set -o pipefail
# Round 5, DMA steps engine: its GPU tests (multi-process parity at P = 2, 3,
# 4, 8, peer killed, thread fallback), then the hand-off cost per dependent
# round next to the host-issued steps and the plan kernel (P = 2, 4).
O=${O:-gpurun_out/r11a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_allreduce_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "dmasteps or dma- or falls_back" > $O/dma_tests.txt 2>&1 || exit 1
run() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2962$1 tools/hop_latency.py > $O/hop_p$1.json 2> $O/hop_p$1.err
}
run 2 4 && run 4 2
