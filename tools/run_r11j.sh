set -o pipefail
# Segmented long reduce streams: the reduce GPU tests (the new segmented case
# included), the N = 1 line at 1 GiB for fp32 / fp16 / bf16, the default
# N = 1 line (256 MiB: one segment), and the segment sweep again.
O=${O:-gpurun_out/r11j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reduce_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/reduce_tests.txt 2>&1 || exit 1
timeout -k 10 300 python tools/seg_1GiB.py > $O/seg.jsonl 2> $O/seg.err || exit 1
timeout -k 10 300 python bench.py --size-mib 1024 --cpu-seconds 2 --no-multidev > $O/bench1_f32_1GiB.json 2> $O/bench1_f32_1GiB.err || exit 1
timeout -k 10 300 python bench.py --dtype f16 --size-mib 1024 --cpu-seconds 5 > $O/bench1_f16_1GiB.json 2> $O/bench1_f16_1GiB.err || exit 1
timeout -k 10 300 python bench.py --dtype bf16 --size-mib 1024 --cpu-seconds 5 > $O/bench1_bf16_1GiB.json 2> $O/bench1_bf16_1GiB.err || exit 1
timeout -k 10 300 python bench.py > $O/bench1.json 2> $O/bench1.err
