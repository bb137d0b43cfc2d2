set -o pipefail
# Request-level HBM counters: read / write
# requests leaving the L2 (TCC_EA0_RDREQ / WRREQ), the part destined for DRAM
# (_DRAM: not served by the memory-side Infinity Cache), the 128-B
# "bubble" requests FETCH_SIZE's formula weighs differently (TCC_BUBBLE), for
# the N = 1 reduce kernel cold (4 buffer pairs) and warm (1 pair), and the
# 8-rank rehearsal's plan kernel at 64 and 256 MiB (rank 0 under --pmc).
mkdir -p gpurun_out/r10d
RD=TCC_EA0_RDREQ,TCC_EA0_RDREQ_DRAM,TCC_BUBBLE
WR=TCC_EA0_WRREQ,TCC_EA0_WRREQ_DRAM,TCC_EA0_WRREQ_64B
N1="bench.py --kernel-only --steps 10 --warmup 2 --no-multidev --no-cpu-baseline --no-staged --no-pmc"
for pairs in 4 1; do
  timeout -s KILL 90 rocprofv3 --pmc $RD --output-format csv -d gpurun_out/r10d/n1rd_p$pairs -o rd -- python3 $N1 --pairs $pairs > gpurun_out/r10d/n1rd_p$pairs.txt 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $WR --output-format csv -d gpurun_out/r10d/n1wr_p$pairs -o wr -- python3 $N1 --pairs $pairs > gpurun_out/r10d/n1wr_p$pairs.txt 2>&1 || exit 1
done
B="bench.py --gpus 8 --steps 20 --warmup 3 --no-sweep --no-staged --no-alt --no-link-probe --candidates ring_chunked --watchdog 240"
export GPU_MAX_HW_QUEUES=1
for mib in 64 256; do
  timeout -k 10 300 python tools/mp_launch.py --nproc 8 --prof-dir gpurun_out/r10d/p8rd_$mib --pmc $RD --prof-name rd -- $B --size-mib $mib > gpurun_out/r10d/p8rd_$mib.json 2> gpurun_out/r10d/p8rd_$mib.err || exit 1
  timeout -k 10 300 python tools/mp_launch.py --nproc 8 --prof-dir gpurun_out/r10d/p8wr_$mib --pmc $WR --prof-name wr -- $B --size-mib $mib > gpurun_out/r10d/p8wr_$mib.json 2> gpurun_out/r10d/p8wr_$mib.err || exit 1
done
