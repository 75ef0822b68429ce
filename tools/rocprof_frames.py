#!/usr/bin/env python3
"""Per-frame spans from a rocprofv3 kernel trace of bench.py.

With heavy tiles a frame is two concurrent launches of trace_simple (the
one-pixel-wave heavy launch on an auxiliary stream, the other tiles on the
launch stream), so no single kernel's average is the frame time.  This groups
the non-counting trace launches into frames (a heavy launch opens a frame; a
frame without one is a single launch) and prints each frame's span, first
start to last end, next to the per-kernel averages.

Usage: python tools/rocprof_frames.py <run_kernel_trace.csv> [--skip N]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=0, help="frames to drop at the start (warmup)")
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if "trace_simple<false, false" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))         # a frame's launches are dispatched together
    frames, cur = [], None
    for r in rows:
        heavy = ", 40, " in r["Kernel_Name"]           # kFeatCoopTail | kFeatFrontier: the heavy launch
        if heavy or cur is None or cur["closed"]:
            cur = {"start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]), "closed": False, "kernels": 0}
            frames.append(cur)
        cur["start"] = min(cur["start"], int(r["Start_Timestamp"]))
        cur["end"] = max(cur["end"], int(r["End_Timestamp"]))
        cur["kernels"] += 1
        if not heavy:
            cur["closed"] = True                        # the other tiles' launch ends a frame
    frames = frames[args.skip:]
    spans = [(f["end"] - f["start"]) / 1e6 for f in frames]
    per_kernel = {}
    for r in rows:
        name = r["Kernel_Name"]
        per_kernel.setdefault(name[name.index("trace_simple"):name.index(">(") + 1], []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(json.dumps({
        "frames": len(spans),
        "frame_span_ms_mean": round(statistics.mean(spans), 4),
        "frame_span_ms_min": round(min(spans), 4),
        "frame_span_ms_max": round(max(spans), 4),
        "launches_per_frame": sorted({f["kernels"] for f in frames}),
        "per_kernel_mean_ms": {k: round(statistics.mean(v), 4) for k, v in per_kernel.items()},
    }, indent=1))


if __name__ == "__main__":
    main()
