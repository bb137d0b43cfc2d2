# round 6: positive controls for the device engines' flag sync
set -o pipefail
O=gpurun_out/r12c; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 170 --timeout-method thread tests/test_sync_control_gpu.py > $O/sync_control_tests.txt 2>&1 || { tail -30 $O/sync_control_tests.txt; exit 1; }
grep -E "PASSED|FAILED" $O/sync_control_tests.txt
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
GLOO_AMD_SYNC=unsafe_noacquire timeout -k 10 300 $L --master-port 29511 bench.py --gpus 4 --steps 5 --warmup 2 --no-sweep --no-staged > $O/bench4_unsafe_noacquire.json 2> $O/bench4_unsafe_noacquire.err || { tail -20 $O/bench4_unsafe_noacquire.err; exit 1; }
timeout -k 10 300 $L --master-port 29512 bench.py --gpus 4 --steps 5 --warmup 2 --no-sweep --no-staged > $O/bench4_narrow.json 2> $O/bench4_narrow.err || { tail -20 $O/bench4_narrow.err; exit 1; }
python - <<'PY'
import json
for f in ("bench4_unsafe_noacquire", "bench4_narrow"):
    d = json.loads(open("gpurun_out/r12c/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d.get("value"), d.get("error"), json.dumps(d.get("device_engines")), {k: (v.get("ok"), v.get("bad_count")) for k, v in d.get("result_checks", {}).items()})
PY
