"""Compact view of convbench logs with '== header' separators (stdin)."""
import json
import sys

for line in sys.stdin:
    if line.startswith("=="):
        print(line.strip())
    elif line.startswith("{"):
        d = json.loads(line)
        if "layer" in d:
            print(f"   {d['layer']:8s}", *[f"{k[:-3]}={d[k]}" for k in ("fwd_us", "dgrad_us", "wgrad_us") if k in d])
        else:
            print("  ", d)
