#!/usr/bin/env python3
"""Device time per frame from a rocprofv3 kernel trace of bench.py.

With D frames in flight the trace launches overlap, so no single kernel's
duration is the frame time.  This takes the timed region's launches (the
last K plain launches of trace_simple before the bench line's
roofline.plain_kernels_after_timed trailing ones (verification, camera stop;
the library counts them, option plain_kernels); counting launches are trace_simple<true, ...> and
learning launches trace_simple<false, true, ...>), and reports:

  union_ms      the union of their [start, end) intervals: time the device
                spent with at least one frame launch running
  span_ms       first start to last end
  per frame     both divided by K
  launches      mean duration (what --stats averages) and the mean number
                running at once (sum of durations / union)

With --bench, the bench.py JSON line of the same run is read and its
ms_per_step (host wall clock per step) is compared with union_ms / K.

Usage: python tools/rocprof_union.py <kernel_trace.csv> --steps K [--bench bench.json] [--out out.json]
"""
import argparse
import csv
import json
import statistics


def union_length(intervals):
    total, cur_s, cur_e = 0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                total += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        total += cur_e - cur_s
    return total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True, help="timed steps (frames) of the bench run")
    ap.add_argument("--launches-per-step", type=int, default=1)
    ap.add_argument("--bench", default="", help="the run's bench.py JSON line (file)")
    ap.add_argument("--out", default="")
    ap.add_argument("--skip-last", type=int, default=-1,
                    help="plain launches after the timed region (default: the bench line's "
                         "roofline.plain_kernels_after_timed, else 0)")
    args = ap.parse_args()
    # plain launches: trace_simple<false, false, ...>
    rows = [r for r in csv.DictReader(open(args.trace)) if "trace_simple<false, false" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    # launches of several frames (bench.py --batch; the N = 1 default is 2):
    # the bench line's config.frames_per_launch
    fpl = 1
    if args.bench:
        line = [x for x in open(args.bench) if x.startswith("{")][-1]
        fpl = int(json.loads(line).get("config", {}).get("frames_per_launch") or 1)
    if args.steps % fpl:
        raise SystemExit(f"{args.steps} frames are not whole launches of {fpl}")
    n = args.steps // fpl * args.launches_per_step
    if len(rows) < n:
        raise SystemExit(f"{len(rows)} plain trace launches in the trace, need {n}")
    skip = args.skip_last
    if args.bench and skip < 0:
        line = [x for x in open(args.bench) if x.startswith("{")][-1]
        skip = json.loads(line).get("roofline", {}).get("plain_kernels_after_timed", 0) or 0
    skip = max(0, skip)
    if len(rows) < n + skip:
        raise SystemExit(f"{len(rows)} plain trace launches in the trace, need {n} + {skip} after them")
    timed = rows[len(rows) - skip - n:len(rows) - skip]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in timed]
    durs = [(e - s) / 1e6 for s, e in iv]
    union = union_length(iv) / 1e6
    span = (max(e for _, e in iv) - min(s for s, _ in iv)) / 1e6
    def short(k):
        return k[k.index("trace_simple"):].split(">(")[0] + ">"
    names = sorted({short(r["Kernel_Name"]) for r in timed})
    by_kernel = {nm: round(statistics.mean((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                                           for r in timed if short(r["Kernel_Name"]) == nm), 4) for nm in names}
    out = {
        "trace": args.trace,
        "kernels": names,
        "mean_ms_by_kernel": by_kernel,
        "frames": args.steps,
        "launches": n,
        "frames_per_launch": fpl,
        "union_ms": round(union, 4),
        "span_ms": round(span, 4),
        "union_ms_per_frame": round(union / args.steps, 4),
        "span_ms_per_frame": round(span / args.steps, 4),
        "launch_ms_mean": round(statistics.mean(durs), 4),
        "launch_ms_min": round(min(durs), 4),
        "launch_ms_max": round(max(durs), 4),
        "launches_in_flight_mean": round(sum(durs) / union, 3),
        # every launch of the production kernel in the trace (settle, warmup,
        # timed, and the 1-frame verification / diagnostic launches after the
        # timed region): what rocprofv3 --stats averages in kernel_stats.csv
        "all_launches": len(rows),
        "all_launch_ms_mean": round(statistics.mean((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                                                    for r in rows), 4),
    }
    if args.bench:
        line = next(ln for ln in open(args.bench) if ln.lstrip().startswith("{"))
        b = json.loads(line)
        out["bench_ms_per_step"] = b["ms_per_step"]
        out["bench_frame_ms_device"] = b.get("roofline", {}).get("frame_ms_device")
        out["bench_kernel_ms"] = b.get("roofline", {}).get("kernel_ms")
        out["union_vs_ms_per_step"] = round(out["union_ms_per_frame"] / b["ms_per_step"], 4)
    text = json.dumps(out, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
