set -o pipefail
# What one device-engine flag poll (a memory-side compare-exchange on
# uncached memory, tools/micro/poll_bytes.hip) adds to each L2->memory
# request counter: K = 0 and K = 1000 polls per workgroup, 512 workgroups.
mkdir -p gpurun_out/r10e
C=TCC_EA0_RDREQ,TCC_EA0_WRREQ,TCC_EA0_ATOMIC,TCC_BUBBLE
for K in 0 1000; do
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r10e/k$K -o poll -- tools/micro/poll_bytes $K 512 > gpurun_out/r10e/k$K.txt 2>&1 || exit 1
done
