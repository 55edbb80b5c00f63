"""One-line summary of a bench.py JSON result (scripts/ab_env.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
deg = d.get("degrid") or {}
c3 = d.get("config3") or {}
print(sys.argv[2], d["value"], d["phases_ms"], deg.get("mvis_s"),
      deg.get("phases_ms"), "c3", c3.get("mvis_s"), c3.get("ms_per_step"),
      c3.get("phases_ms"))
