#!/usr/bin/env python3
"""Table of tools/emulate.sh results (one bench.py JSON per emulated rank):
per run tag the slowest rank's ms per step and the speedup over a one-GPU
bench.py JSON of the same box.  Usage: emu_summary.py DIR BASE_JSON [BASE200_JSON]"""
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(f):
    lines = [x for x in open(f) if x.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main():
    d, base = sys.argv[1], load(sys.argv[2])
    base200 = load(sys.argv[3]) if len(sys.argv) > 3 else None
    runs = defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        m = re.match(r"(.*)_n(\d+)_r(\d+)\.json$", os.path.basename(f))
        j = load(f)
        if m and j:
            runs[(m.group(1), int(m.group(2)))][int(m.group(3))] = j
    for (tag, n), ranks in sorted(runs.items()):
        b = base200 if ("200" in tag and base200) else base
        worst = max(ranks.values(), key=lambda j: j["ms_per_step"])
        c = worst["config"]
        per = {r: round(j["ms_per_step"], 4) for r, j in sorted(ranks.items())}
        # a step is frames_per_step frames: the N-GPU rate if every rank ran at the slowest one's pace
        rate = worst["value"]
        print(json.dumps({"tag": tag, "N": n, "scaling": worst["scaling"], "steps": worst["steps"],
                          "frames_per_launch": c["frames_per_launch"], "launches_in_flight": c["launches_in_flight"],
                          "exchange_every": c["exchange_every_frames"], "root_weight": c["root_weight"],
                          "ms_per_step_by_rank": per, "job_mrays_s": rate,
                          "one_gpu_mrays_s": b["value"], "speedup": round(rate / b["value"], 2)}))


if __name__ == "__main__":
    main()
