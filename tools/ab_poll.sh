#!/bin/bash
# A/B of the plan kernel's flag polls: compare-exchange (default) vs
# system-scope loads (GLOO_AMD_POLL=load).  Correctness under load polls
# first (the sync-control soaks and the device-engine fuzz), then hop latency
# at P = 2, 4, 8 and the 8-rank 256 MiB ring, alternating the two.
set -o pipefail
O=${O:-gpurun_out/ab_poll}
mkdir -p "$O"
export TMPDIR=/tmp
GLOO_AMD_POLL=load timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/test_sync_control_gpu.py tests/test_fuzz_gpu.py \
  -k "soak_exact or catches or random_cases_multiprocess" > "$O/tests_load.txt" 2>&1 || { tail -5 "$O/tests_load.txt"; exit 1; }
tail -1 "$O/tests_load.txt"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for v in cas load cas load; do
  for pq in "2 4" "4 2" "8 1"; do
    set -- $pq
    GLOO_AMD_POLL=$v GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 $TR --nproc-per-node $1 \
      --master-port 2958$1 tools/hop_latency.py --engines plan_kernel --iters 300 \
      >> "$O/hop_$v.jsonl" 2>> "$O/hop.err" || exit 1
  done
done
for v in cas load; do
  GLOO_AMD_POLL=$v GPU_MAX_HW_QUEUES=1 timeout -k 10 400 $TR --nproc-per-node 8 --master-port 29591 \
    bench.py --gpus 8 --candidates ring_chunked --no-alt --no-link-probe --no-sweep --no-staged \
    --steps 20 --warmup 3 > "$O/mp8_$v.json" 2> "$O/mp8_$v.err" || exit 1
done
echo done
