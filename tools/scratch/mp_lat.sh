#!/bin/bash
# usage: mp_lat.sh P mode tag  -> gpurun_out/lat_<tag>_r<rank>.log (one process per rank)
P=$1; MODE=$2; TAG=$3
D=$(mktemp -d)
pids=()
for r in $(seq 0 $((P-1))); do
  python tests/mp_worker.py $D $r $P $MODE > gpurun_out/lat_${TAG}_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
grep -h "^LAT" gpurun_out/lat_${TAG}_r0.log
exit $rc
