"""Print the key fields of a bench.py JSON line (reads the log on stdin)."""
import json
import sys

for line in sys.stdin:
    if line.startswith("{"):
        d = json.loads(line)
        r = d.get("roofline") or {}
        print("BENCH", d["value"], "img/s", d["ms_per_step"], "ms/step  host", d.get("host_issue_ms_per_step"),
              "ms  util", d["mfma_util_step"], r.get("families_avg_ms"))
