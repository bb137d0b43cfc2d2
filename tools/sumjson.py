"""Summarise bench.py JSON lines (N>1): value, schedule/engine, alternatives, sweep."""
import faulthandler
import json
import sys

faulthandler.enable()  # a crash prints every thread's stack

for f in sys.argv[1:]:
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no JSON")
        continue
    d = json.loads(lines[-1])
    c = d["config"]
    print(f, "value", d["value"], "ms", d["ms_per_step"], c.get("schedule"), c.get("engine"),
          c.get("transport"), "verified", d.get("verified"))
    for a, v in (d.get("alt_schedules") or {}).items():
        print("   alt", a, v.get("engine"), v["ms_per_step"], "ms", v["value"])
    for n, row in (d.get("sweep") or {}).items():
        print("   ", n, {k: (v["us"], v.get("engine", "")) for k, v in row.items()})
