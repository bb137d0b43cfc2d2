set -o pipefail
# End of round 5: full GPU suite, smoke(), then the bench records -- the N = 1
# default line, configs[4]'s element types at 1 GiB (N = 1: the reduce kernel
# on f16 / bf16), the same N = 1 command under rocprofv3, and the N > 1
# rehearsals at P = 8, 4, 2 (ranks sharing the box's GPU, default flags).
O=${O:-gpurun_out/r11f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=40 > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench1.json 2> $O/bench1.err || exit 1
timeout -k 10 300 python bench.py --dtype f16 --size-mib 1024 --cpu-seconds 5 > $O/bench1_f16_1GiB.json 2> $O/bench1_f16_1GiB.err || exit 1
timeout -k 10 300 python bench.py --dtype bf16 --size-mib 1024 --cpu-seconds 5 > $O/bench1_bf16_1GiB.json 2> $O/bench1_bf16_1GiB.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1prof -o n1 -- python3 bench.py --no-pmc > $O/bench1_under_rocprof.json 2> $O/bench1_under_rocprof.err || exit 1
run() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2953$1 bench.py --gpus $1 > $O/mp$1_shared_gpu.json 2> $O/mp$1_shared_gpu.err
}
run 8 1 && run 4 2 && run 2 4
