"""The value and the dominant kernel's launch time of the legs named in FIELD (space-separated; default the
headline) from the last JSON line of a bench.py run on stdin (scripts/gpu_ab.sh)."""
import json
import os
import sys

d = [json.loads(x) for x in sys.stdin if x.startswith("{")][-1]
out = []
for f in os.environ.get("FIELD", "").split() or [""]:
    e = d[f] if f and f != "headline" else d
    out.append(f"{f or 'headline'} {e['value']:.0f} {e['roofline']['mean_launch_us']:.1f}")
print("  ".join(out))
