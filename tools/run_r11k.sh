set -o pipefail
# configs[4]'s 1 GiB N = 1 lines after the reduce launches were segmented
# (fp32 / fp16 / bf16, live PMC traffic per call), and fp16 under rocprofv3
# (four dispatches per call).
O=${O:-gpurun_out/r11k}
mkdir -p $O
export TMPDIR=/tmp
for d in f32 f16 bf16; do
  timeout -k 10 300 python bench.py --dtype $d --size-mib 1024 --cpu-seconds 5 > $O/bench1_${d}_1GiB.json 2> $O/bench1_${d}_1GiB.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f16prof -o f16 -- python3 bench.py --dtype f16 --size-mib 1024 --no-pmc --cpu-seconds 2 > $O/bench1_f16_1GiB_under_rocprof.json 2> $O/bench1_f16_1GiB_under_rocprof.err
