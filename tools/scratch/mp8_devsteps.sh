#!/bin/bash
# 8 processes of `mp_worker.py devsteps` on this GPU from tree $1 (the
# round-1 library or the current one); logs to gpurun_out/$2.r<k>.log.
set -u
TREE=$1; TAG=$2
D=$(mktemp -d)
pids=()
for r in 0 1 2 3 4 5 6 7; do
  (cd "$TREE" && HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 360 python -u tests/mp_worker.py "$D" $r 8 devsteps) \
    > "gpurun_out/$TAG.r$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
grep -h "MISMATCH\|Timed out\|^OK" gpurun_out/$TAG.r*.log | head -20
exit $rc
