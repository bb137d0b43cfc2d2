set -o pipefail
# IPC import of allocations around 2 GiB (the two-shot mesh's slot arrays at
# count INT_MAX int8 hung in resolvePeers).
O=${O:-gpurun_out/r11x}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
D=$(mktemp -d)
timeout -k 5 60 python -u tools/micro/ipc_size_probe.py export $D $FLAGS > $O/${TAG}export.txt 2>&1 &
E=$!
timeout -k 5 60 python -u tools/micro/ipc_size_probe.py import $D > $O/${TAG}import.txt 2>&1
rc=$?
wait $E || rc=$?
rm -rf $D
exit $rc
