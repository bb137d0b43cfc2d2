set -o pipefail
# After the per-workgroup launch counters: every device-engine GPU test that
# exercises them (graph capture + overlap, soak, multi-process engines,
# fuzz), then tools/hop_latency.py at P = 2, 4, 8, then the widening suite.
O=gpurun_out/r10k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_graph_capture_gpu.py tests/test_soak_gpu.py tests/test_fuzz_gpu.py "tests/test_allreduce_gpu.py::test_device_engine_multiprocess" "tests/test_allreduce_gpu.py::test_peer_killed_raises_io_exception" "tests/test_allreduce_gpu.py::test_device_engine_timeout_raises_io_exception" > $O/devengine_tests.txt 2>&1 || exit 1
run() {  # P queues
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 2952$1 tools/hop_latency.py > $O/hop_p$1.json 2> $O/hop_p$1.err
}
run 2 4 && run 4 2 && run 8 1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m widening -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/widening_suite.txt 2>&1
