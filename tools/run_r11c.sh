set -o pipefail
# Timeline of the DMA steps engine's ring: P = 2 ranks on the box's GPU, rank 0
# under rocprofv3 (kernels and memory copies), 1 M floats and 64 M floats
# (the north-star size) per rank.
O=${O:-gpurun_out/r11c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/mp_launch.py --nproc 2 --port 29631 --prof-dir $O/p2 --prof-name dma --copies -- tools/hop_latency.py --sizes 1048576,67108864 --iters 20 --engines dma_steps,host_steps > $O/p2.json 2> $O/p2.err
