set -o pipefail
O=gpurun_out/r12f; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 350 --timeout-method thread tests/test_scale_gpu.py::test_max_int_count_every_engine > $O/maxcount.txt 2>&1 || { grep -E "maxcount rank 0|FAILED" $O/maxcount.txt | tail -30; exit 1; }
grep -E "maxcount rank 0.*(ok|MISMATCH|refused)" $O/maxcount.txt
timeout -k 10 700 python -u -m pytest -q -x --timeout 170 --timeout-method thread tests/test_allreduce_gpu.py tests/test_allreduce_fn_gpu.py tests/test_host_endpoints_gpu.py tests/test_allreduce_custom.py tests/test_reference_binding.py > $O/suite_part.txt 2>&1; rc=$?
tail -3 $O/suite_part.txt; exit $rc
