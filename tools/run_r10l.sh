set -o pipefail
# Where the host-issued ring's time per round goes: P = 2 ranks on the box's
# GPU, 1K floats, host-issued steps only, rank 0 under rocprofv3 with kernel,
# memory-copy and HIP runtime traces (tools/hop_latency.py, tools/mp_launch.py).
O=gpurun_out/r10l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/mp_launch.py --nproc 2 --port 29611 --prof-dir $O/p2 --prof-name host --copies --api -- tools/hop_latency.py --sizes 1024 --iters 100 --engines host_steps > $O/p2.json 2> $O/p2.err
