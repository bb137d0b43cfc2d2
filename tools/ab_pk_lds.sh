set -o pipefail; O=gpurun_out/r12l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_fuzz_gpu.py tests/test_graph_capture_gpu.py tests/test_sync_control_gpu.py "tests/test_scale_gpu.py::test_north_star_size_vs_reference" > $O/tests.txt 2>&1 || { tail -5 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in 0 1 0 1; do
  for pq in "2 4" "4 2" "8 1"; do set -- $pq
    GLOO_AMD_PK_LDS=$v GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node $1 --master-port 2957$1 tools/hop_latency.py --engines plan_kernel --iters 300 >> $O/hop_lds$v.jsonl 2>> $O/hop.err || exit 1
  done
done
for v in 0 1; do
  GLOO_AMD_PK_LDS=$v GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 8 --master-port 29581 bench.py --gpus 8 --candidates ring_chunked --no-alt --no-link-probe --no-sweep --no-staged --steps 20 --warmup 3 > $O/mp8_lds$v.json 2> $O/mp8_lds$v.err || exit 1
done
echo done
