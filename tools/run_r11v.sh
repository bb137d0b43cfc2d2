set -o pipefail
# The max-count (INT_MAX elements) worker at P = 2, each rank's output
# straight to a file (the pytest wrapper holds it until the end).
O=${O:-gpurun_out/r11v}
mkdir -p $O
D=$(mktemp -d)
export HSA_ENABLE_IPC_MODE_LEGACY=0 GLOO_AMD_DEVICE_ENGINES=shared
for r in 0 1; do
  timeout -k 10 280 python -u tests/mp_worker.py $D $r 2 maxcount > $O/rank$r.txt 2>&1 &
done
rc=0
for j in $(jobs -p); do wait $j || rc=$?; done
rm -rf $D
exit $rc
