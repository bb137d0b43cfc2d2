set -o pipefail
# The reduce kernel on the HBM-only loop at configs[4]'s 1 GiB: launch shape and
# cache policy sweeps for fp16, bf16 and fp32 (is the 16-bit line's lower
# fraction the element type or the size?).
O=${O:-gpurun_out/r11h}
mkdir -p $O
timeout -k 10 300 python tools/tune_cold.py 1024 f32 > $O/tune_cold_f32_1GiB.jsonl 2> $O/f32.err || exit 1
timeout -k 10 300 python tools/tune_cold.py 1024 f16 > $O/tune_cold_f16_1GiB.jsonl 2> $O/f16.err || exit 1
timeout -k 10 300 python tools/tune_cold.py 1024 bf16 > $O/tune_cold_bf16_1GiB.jsonl 2> $O/bf16.err
