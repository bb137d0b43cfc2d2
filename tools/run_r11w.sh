set -o pipefail
# Diagnose the two-shot mesh at count INT_MAX (int8): 1 GiB first, then the
# full count, 20 s context timeout, each rank under its own time limit.
O=${O:-gpurun_out/r11w}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 GLOO_AMD_DEVICE_ENGINES=shared MAXCOUNT_SCHED=mesh \
  MAXCOUNT_DTYPE=int8 MAXCOUNT_TIMEOUT=20 GLOO_AMD_TRACE=1 GLOO_AMD_TRACE_MEM=1
for N in ${NS:-1073741827 2147483647}; do
  D=$(mktemp -d)
  for r in 0 1; do
    MAXCOUNT_N=$N timeout -k 10 60 python -u tests/mp_worker.py $D $r 2 maxcount > $O/n${N}_rank$r.txt 2>&1 &
  done
  rc=0
  for j in $(jobs -p); do wait $j || rc=$?; done
  rm -rf $D
  echo "N=$N rc=$rc" >> $O/summary.txt
  [ $rc -eq 0 ] || exit $rc
done
