set -o pipefail
# DMA steps engine with one copy stream per channel: its GPU tests, the
# hand-off per round (P = 2, 4) and the three rings at 256 MiB (P = 2, 4, 8).
O=${O:-gpurun_out/r11e}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_allreduce_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "dmasteps or dma- or falls_back" > $O/dma_tests.txt 2>&1 || exit 1
hop() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2991$1 tools/hop_latency.py > $O/hop_p$1.json 2> $O/hop_p$1.err
}
rings() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2992$1 bench.py --gpus $1 --candidates ring_chunked,ring_chunked_host,ring_chunked_dma --no-alt --no-link-probe --no-sweep --no-staged --steps 10 --warmup 3 > $O/mp$1_rings.json 2> $O/mp$1_rings.err
}
hop 2 4 && hop 4 2 && rings 2 4 && rings 4 2 && rings 8 1
