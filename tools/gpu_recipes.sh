#!/bin/bash
# The GPU session recipes behind the records in profiles/ (one parametrised
# runner; replaces round 5's 22 one-off tools/run_r1*.sh scripts).  Run on
# the GPU box, e.g.
#   gpurun -- 'O=gpurun_out/x bash tools/gpu_recipes.sh suite smoke bench1'
# Every step has its own time limit; the first failing step ends the call
# (nothing further runs on the GPU after a failure, a fault or a time limit).
#
#   suite              pytest -m gpu (durations) -> $O/gpu_suite.txt
#   smoke              __graft_entry__.smoke()   -> $O/smoke.txt
#   bench1             bench.py (N = 1, default)  -> $O/bench1.json
#   bench1_1gib        configs[4]: fp32 / fp16 / bf16 at 1 GiB -> $O/bench1_<d>_1GiB.json
#   bench1_rocprof     bench.py --no-pmc under rocprofv3 --kernel-trace --stats -> $O/n1prof
#   rehearsals         bench.py --gpus P at P = 8, 4, 2 (ranks share the GPU) -> $O/mp<P>_shared_gpu.json
#   rings              the three rings at 256 MiB, P = 2, 4, 8 -> $O/mp<P>_rings.json
#   pipe               the rings with and without pipelining below chunk granularity, P = 2
#                      at piece sizes $PIPES (MiB, default "1 4 16"), P = 4, 8 at 4 MiB
#                      -> $O/pipe_p<P>_<MiB>MiB.json
#   hop                tools/hop_latency.py at P = 2, 4 (ENGINES=...) -> $O/hop_p<P>.json
#   dma_tests          the DMA steps engine's GPU tests -> $O/dma_tests.txt
#   soak               tests/test_soak_gpu.py -> $O/soak.txt
#   tune_cold          tools/tune_cold.py at 1 GiB, f32 / f16 / bf16 -> $O/tune_cold_<d>_1GiB.jsonl
#   segments           tools/seg_1GiB.py and tools/seg_fold.py -> $O/seg*.jsonl
#   maxcount           the INT_MAX-count worker at P = 2, each rank to a file -> $O/rank<r>.txt
#   sync_control       tools/sync_control.py P = 2, 4, 8 at 4096 elements -> $O/sync_control.json
#   ipc_probe          tools/micro/ipc_size_probe.py export / import (FLAGS, TAG) -> $O/*port.txt
#   timeline           rank 0 of a P = 2 hop_latency run under rocprofv3 (ENGINES) -> $O/p2
set -o pipefail
O=${O:-gpurun_out/recipes}
mkdir -p "$O"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python -u -m pytest --timeout 300 --timeout-method thread -p no:cacheprovider"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"

mp() {  # P queues port args... -> torchrun of bench.py on the shared GPU
  local P=$1 q=$2 port=$3
  shift 3
  GPU_MAX_HW_QUEUES=$q timeout -k 10 600 $TR --nproc-per-node "$P" --master-port "$port" \
    bench.py --gpus "$P" "$@"
}

recipe() {
  case "$1" in
    suite) timeout -k 10 900 $PYT tests -m gpu -q --durations=40 > "$O/gpu_suite.txt" 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" \
             > "$O/smoke.txt" 2>&1 ;;
    bench1) timeout -k 10 300 python bench.py > "$O/bench1.json" 2> "$O/bench1.err" ;;
    bench1_1gib)
      for d in f32 f16 bf16; do
        timeout -k 10 300 python bench.py --dtype $d --size-mib 1024 --cpu-seconds 5 \
          > "$O/bench1_${d}_1GiB.json" 2> "$O/bench1_${d}_1GiB.err" || return 1
      done ;;
    bench1_rocprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/n1prof" -o n1 \
        -- python3 bench.py --no-pmc > "$O/bench1_under_rocprof.json" 2> "$O/bench1_under_rocprof.err" ;;
    rehearsals)
      mp 8 1 29531 > "$O/mp8_shared_gpu.json" 2> "$O/mp8_shared_gpu.err" &&
        mp 4 2 29532 > "$O/mp4_shared_gpu.json" 2> "$O/mp4_shared_gpu.err" &&
        mp 2 4 29533 > "$O/mp2_shared_gpu.json" 2> "$O/mp2_shared_gpu.err" ;;
    rings)
      local a="--candidates ring_chunked,ring_chunked_host,ring_chunked_dma --no-alt --no-link-probe"
      a="$a --no-sweep --no-staged --steps 10 --warmup 3"
      mp 2 4 29541 $a > "$O/mp2_rings.json" 2> "$O/mp2_rings.err" &&
        mp 4 2 29542 $a > "$O/mp4_rings.json" 2> "$O/mp4_rings.err" &&
        mp 8 1 29543 $a > "$O/mp8_rings.json" 2> "$O/mp8_rings.err" ;;
    pipe)
      local a="--candidates ring_chunked,ring_chunked_host,ring_chunked_host_pipe"
      a="$a,ring_chunked_dma,ring_chunked_dma_pipe --no-alt --no-link-probe --no-sweep --no-staged"
      a="$a --steps 10 --warmup 3"
      for m in ${PIPES:-1 4 16}; do
        BENCH_PIPE_BYTES=$((m << 20)) mp 2 4 29561 $a > "$O/pipe_p2_${m}MiB.json" \
          2> "$O/pipe_p2_${m}MiB.err" || return 1
      done
      BENCH_PIPE_BYTES=$((4 << 20)) mp 4 2 29562 $a > "$O/pipe_p4_4MiB.json" 2> "$O/pipe_p4_4MiB.err" &&
        BENCH_PIPE_BYTES=$((4 << 20)) mp 8 1 29563 $a > "$O/pipe_p8_4MiB.json" 2> "$O/pipe_p8_4MiB.err" ;;
    hop)
      for pq in "2 4" "4 2"; do
        set -- $pq
        GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 $TR --nproc-per-node $1 --master-port 2955$1 \
          tools/hop_latency.py ${ENGINES:+--engines $ENGINES} > "$O/hop_p$1.json" \
          2> "$O/hop_p$1.err" || return 1
      done ;;
    dma_tests) timeout -k 10 900 $PYT tests/test_allreduce_gpu.py -x -v \
                 -k "dmasteps or dma- or falls_back or dma_steps" > "$O/dma_tests.txt" 2>&1 ;;
    soak) timeout -k 10 900 $PYT tests/test_soak_gpu.py -x -v > "$O/soak.txt" 2>&1 ;;
    tune_cold)
      for d in f32 f16 bf16; do
        timeout -k 10 300 python tools/tune_cold.py 1024 $d > "$O/tune_cold_${d}_1GiB.jsonl" \
          2> "$O/tune_cold_$d.err" || return 1
      done ;;
    segments)
      timeout -k 10 300 python tools/seg_1GiB.py > "$O/seg.jsonl" 2> "$O/seg.err" &&
        timeout -k 10 200 python tools/seg_fold.py > "$O/seg_fold.jsonl" 2> "$O/seg_fold.err" ;;
    maxcount)
      local D rc=0
      D=$(mktemp -d)
      for r in 0 1; do
        GLOO_AMD_DEVICE_ENGINES=shared timeout -k 10 280 python -u tests/mp_worker.py "$D" $r 2 \
          maxcount > "$O/rank$r.txt" 2>&1 &
      done
      for j in $(jobs -p); do wait "$j" || rc=$?; done
      rm -rf "$D"
      return $rc ;;
    sync_control) timeout -k 10 600 python -u tools/sync_control.py "$O/sync_control.json" \
                    --runs 200 --P 2,4,8 --n 4096 > "$O/sync_control.log" 2>&1 ;;
    ipc_probe)
      local D E rc
      D=$(mktemp -d)
      timeout -k 5 60 python -u tools/micro/ipc_size_probe.py export "$D" $FLAGS \
        > "$O/${TAG}export.txt" 2>&1 &
      E=$!
      timeout -k 5 60 python -u tools/micro/ipc_size_probe.py import "$D" > "$O/${TAG}import.txt" 2>&1
      rc=$?
      wait $E || rc=$?
      rm -rf "$D"
      return $rc ;;
    timeline) timeout -k 10 300 python tools/mp_launch.py --nproc 2 --port 29651 --prof-dir "$O/p2" \
                --prof-name ${PROF_NAME:-hop} --copies -- tools/hop_latency.py \
                --sizes ${SIZES:-1048576} --iters 20 ${ENGINES:+--engines $ENGINES} \
                > "$O/p2.json" 2> "$O/p2.err" ;;
    *) echo "unknown recipe $1" >&2; return 2 ;;
  esac
}

for r in "$@"; do
  echo "[recipes] $r -> $O" >&2
  recipe "$r" || { echo "[recipes] $r failed (rc $?); stopping" >&2; exit 1; }
done
