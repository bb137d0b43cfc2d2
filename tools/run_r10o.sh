set -o pipefail
# Timeline of the host-issued ring with P = 2 rank THREADS (no other process
# on the GPU): kernel, memory-copy and HIP API traces of the whole process.
O=gpurun_out/r10o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $O/t2 -o thr -- python3 tools/hop_latency_threads.py --ranks 2 --sizes 1024 --iters 100 > $O/t2.json 2> $O/t2.err
