set -o pipefail
# The soak tests with the DMA steps engine's ring and halving-doubling added
# (every mode, the round-4 failure configuration included).
O=${O:-gpurun_out/r11q}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_soak_gpu.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/soak.txt 2>&1
