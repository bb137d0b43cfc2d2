set -o pipefail
# Experiment (its switch since removed): the DMA steps engine's post-copy signals as hipStreamWriteValue64
# (GLOO_AMD_DMA_WRITE_VALUE=1) instead of a flag kernel: the engine's GPU test
# at P = 2 and 3, the hand-off per round at P = 2 and the rings at P = 2;
# rank 0's trace at P = 2.
O=${O:-gpurun_out/r11g}
mkdir -p $O
export TMPDIR=/tmp
export GLOO_AMD_DMA_WRITE_VALUE=1
timeout -k 10 600 python -u -m pytest tests/test_allreduce_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "multiprocess and dmasteps and (2- or 3-)" > $O/dma_tests.txt 2>&1 || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29942 tools/hop_latency.py --engines host_steps,dma_steps > $O/hop_p2.json 2> $O/hop_p2.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29952 bench.py --gpus 2 --candidates ring_chunked,ring_chunked_host,ring_chunked_dma --no-alt --no-link-probe --no-sweep --no-staged --steps 10 --warmup 3 > $O/mp2_rings.json 2> $O/mp2_rings.err || exit 1
timeout -k 10 300 python tools/mp_launch.py --nproc 2 --port 29643 --prof-dir $O/p2 --prof-name dma --copies -- tools/hop_latency.py --sizes 1048576,67108864 --iters 20 --engines dma_steps,host_steps > $O/p2.json 2> $O/p2.err
