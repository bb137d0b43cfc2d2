set -o pipefail
# Attribution of the plan kernel's HBM excess over its algorithmic bytes (VERDICT r4
# #5): the 8-rank shared-GPU rehearsal, rank 0 under rocprofv3 --pmc, at two sizes,
# with the flag polls counted (GLOO_AMD_COUNT_POLLS=1); the counter list of the box.
mkdir -p gpurun_out/r10c
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r10c/counters.txt 2>&1 || true
B="bench.py --gpus 8 --steps 20 --warmup 3 --no-sweep --no-staged --no-alt --no-link-probe --candidates ring_chunked --watchdog 240"
export GLOO_AMD_COUNT_POLLS=1 GPU_MAX_HW_QUEUES=1
timeout -k 10 300 python tools/mp_launch.py --nproc 8 --prof-dir gpurun_out/r10c/f64 --pmc FETCH_SIZE --prof-name fetch -- $B --size-mib 64 > gpurun_out/r10c/f64.json 2> gpurun_out/r10c/f64.err &&
timeout -k 10 300 python tools/mp_launch.py --nproc 8 --prof-dir gpurun_out/r10c/w64 --pmc WRITE_SIZE --prof-name write -- $B --size-mib 64 > gpurun_out/r10c/w64.json 2> gpurun_out/r10c/w64.err &&
timeout -k 10 300 python tools/mp_launch.py --nproc 8 --prof-dir gpurun_out/r10c/w256 --pmc WRITE_SIZE --prof-name write -- $B > gpurun_out/r10c/w256.json 2> gpurun_out/r10c/w256.err &&
timeout -k 10 300 python tools/mp_launch.py --nproc 8 --prof-dir gpurun_out/r10c/rq256 --pmc TCC_EA0_RDREQ,TCC_EA0_RDREQ_32B --prof-name rq -- $B > gpurun_out/r10c/rq256.json 2> gpurun_out/r10c/rq256.err
