set -o pipefail
# Round-5 bench records: the N = 1 default line, the same command under
# rocprofv3 --kernel-trace --stats (rocprof's per-launch time of the timed
# loop vs the bench's HIP events; --no-pmc: no profiler children inside the
# profiled process), and the N > 1 rehearsals (ranks sharing the box's one
# GPU, torchrun as the driver launches it) at P = 8, 4, 2.
O=${O:-gpurun_out/r10g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench1.json 2> $O/bench1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1prof -o n1 -- python3 bench.py --no-pmc > $O/bench1_under_rocprof.json 2> $O/bench1_under_rocprof.err || exit 1
run() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2951$1 bench.py --gpus $1 > $O/mp$1_shared_gpu.json 2> $O/mp$1_shared_gpu.err
}
run 8 1 || exit 1
run 4 2 || exit 1
run 2 4 || exit 1
