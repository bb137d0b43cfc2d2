set -o pipefail
# The fold kernel's segmented launches: the reduce GPU tests and the fold
# measurement again (one call is now segmented inside the library).
O=${O:-gpurun_out/r11m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reduce_gpu.py tests/test_allreduce_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "reduce or multi_pointer or fold" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 200 python tools/seg_fold.py > $O/seg_fold.jsonl 2> $O/seg_fold.err
