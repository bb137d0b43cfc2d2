set -o pipefail
# The DMA steps engine with the runtime's copies on blit kernels instead of
# the SDMA engines (HSA_ENABLE_SDMA=0): hand-off cost per round at P = 2, 4
# and the three rings at 256 MiB at P = 2, 4, 8 on the box's one GPU.
O=${O:-gpurun_out/r11d}
mkdir -p $O
export HSA_ENABLE_SDMA=0
hop() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2981$1 tools/hop_latency.py --engines host_steps,dma_steps > $O/hop_p$1.json 2> $O/hop_p$1.err
}
rings() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2982$1 bench.py --gpus $1 --candidates ring_chunked,ring_chunked_host,ring_chunked_dma --no-alt --no-link-probe --no-sweep --no-staged --steps 10 --warmup 3 > $O/mp$1_rings.json 2> $O/mp$1_rings.err
}
hop 2 4 && hop 4 2 && rings 2 4 && rings 4 2 && rings 8 1
