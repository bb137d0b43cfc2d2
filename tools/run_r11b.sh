set -o pipefail
# The three rings at the north-star size on the one-GPU box (ranks sharing
# it): plan kernel, host-issued DMA steps, DMA steps with on-GPU hand-offs.
O=${O:-gpurun_out/r11b}
mkdir -p $O
run() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2971$1 bench.py --gpus $1 --candidates ring_chunked,ring_chunked_host,ring_chunked_dma --no-alt --no-link-probe --no-sweep --no-staged --steps 10 --warmup 3 > $O/mp$1_rings.json 2> $O/mp$1_rings.err
}
run 2 4 && run 4 2 && run 8 1
