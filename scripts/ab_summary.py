"""One-line summary of a bench.py JSON result (scripts/ab_env.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
deg = d.get("degrid") or {}
print(sys.argv[2], d["value"], d["phases_ms"], deg.get("mvis_s"),
      deg.get("phases_ms"))
