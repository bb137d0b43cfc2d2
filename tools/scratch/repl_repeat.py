"""Repeat test_replicated_schedule_matches_ring_chunked_oracle(P, N) and count
wrong results, under the copy engine named on the command line."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))

import gloo_amd  # noqa: E402
import test_allreduce_gpu as T  # noqa: E402

engine = sys.argv[1]
reps = int(sys.argv[2])
cases = [(8, 100003), (8, 4099), (4, 100003), (3, 100003)]
gloo_amd.set_copy_engine(engine, 64)
bad = 0
for rep in range(reps):
    for P, N in cases:
        try:
            T.test_replicated_schedule_matches_ring_chunked_oracle(P, N)
        except AssertionError as e:
            bad += 1
            print("rep %d P %d N %d: MISMATCH %s" % (rep, P, N, str(e).splitlines()[0][:120]),
                  flush=True)
print("engine %s: %d wrong of %d" % (engine, bad, reps * len(cases)), flush=True)
