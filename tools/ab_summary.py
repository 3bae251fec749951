"""Summarise gpurun_out/ab.log (tools/gpu.sh ab): ms/step per knob setting."""
import collections
import json
import sys

cur, r = None, collections.defaultdict(list)
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    if line.startswith("=="):
        cur = line[3:].strip()
    elif line.startswith("{") and '"metric"' in line:
        r[cur].append(json.loads(line)["ms_per_step"])
for k, v in r.items():
    print(f"{k:28s} mean {sum(v) / len(v):.3f} ms  {v}")
