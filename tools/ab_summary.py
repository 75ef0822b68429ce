#!/usr/bin/env python3
"""Summarise tools/session_ab.sh results: ms/frame per arm."""
import glob
import json
import os
import re
import sys

d = sys.argv[1]
arms = {}
for f in sorted(glob.glob(os.path.join(d, "bench_a*_*.json"))):
    m = re.search(r"bench_a(\d+)_(\d+)\.json", f)
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        continue
    j = json.loads(lines[-1])
    arms.setdefault(int(m.group(1)), []).append((j["ms_per_step"], j["value"], j["config"]["schedule"].get("heavy_tiles_used")))
for k in sorted(arms):
    print(k, " ".join(f"{ms:.4f}ms/{v:.0f}({h})" for ms, v, h in arms[k]))
